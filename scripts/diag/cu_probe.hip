// cu_probe.hip (diagnostic): which XCC / SE / CU each workgroup of a launch runs on, to check how
// a hipExtStreamCreateWithCUMask mask maps onto the chip.  Build: scripts/diag/build_cu_probe.sh
#include <hip/hip_runtime.h>

__global__ void k_cu_probe(int* out, int spin) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    // keep the workgroup resident for a while so the launch spreads over every allowed CU
    long long t0 = clock64();
    while (clock64() - t0 < spin) {}
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = (int)hw;
        out[2 * blockIdx.x + 1] = (int)xcc;
    }
}

extern "C" int cu_probe(int* out, int n_wg, int spin, void* stream) {
    hipLaunchKernelGGL(k_cu_probe, dim3(n_wg), dim3(64), 0, (hipStream_t)stream, out, spin);
    return (int)hipGetLastError();
}
