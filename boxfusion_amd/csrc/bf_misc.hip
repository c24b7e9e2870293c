// bf_misc.hip — library identity
#include "bf_common.h"

BF_API const char* bf_version(void) { return "boxfusion_hip 0.1.0 gfx950"; }

BF_API int bf_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

// ------------------------------------------------------------------------------------------
// bf_rows_gather: every field of a box set gathered / concatenated in one launch.
// blockIdx.y = field; threads stride over (row, 4-byte word) of that field's output.
// ------------------------------------------------------------------------------------------
struct RowsArgs {
    bf_rows_field f[BF_ROWS_MAX_FIELDS];
};

__global__ void __launch_bounds__(256) k_rows_gather(RowsArgs args, const void* __restrict__ idx,
                                                     int idx_i32, int n_out, int32_t* __restrict__ status) {
    const bf_rows_field& F = args.f[blockIdx.y];
    const bool narrow = F.pad == 1;                       // int64 source rows -> int32 output
    const int wpr = narrow ? F.row_bytes >> 3 : F.row_bytes >> 2;   // output words per row
    const long long total = (long long)n_out * wpr;
    const long long na = F.n_a, nab = F.n_a + F.n_b;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (long long)gridDim.x * blockDim.x) {
        const long long r = e / wpr, w = e - r * wpr;
        const long long s = !idx ? r : idx_i32 ? (long long)static_cast<const int32_t*>(idx)[r]
                                               : static_cast<const int64_t*>(idx)[r];
        if (s < 0 || s >= nab) {
            if (status && w == 0) atomicOr(status, BF_DEV_INDEX_RANGE);
            continue;
        }
        if (narrow) {
            const int64_t* src = s < na ? static_cast<const int64_t*>(F.a) + s * wpr
                                        : static_cast<const int64_t*>(F.b) + (s - na) * wpr;
            static_cast<int32_t*>(F.dst)[e] = (int32_t)src[w];
            continue;
        }
        const uint32_t* src = s < na ? static_cast<const uint32_t*>(F.a) + s * wpr
                                     : static_cast<const uint32_t*>(F.b) + (s - na) * wpr;
        static_cast<uint32_t*>(F.dst)[e] = src[w];
    }
}

BF_API int bf_rows_gather(const bf_rows_field* fields, int n_fields, const void* idx, int idx_i32,
                          int n_out, int32_t* status, void* stream) {
    if (!fields || n_fields < 0 || n_fields > BF_ROWS_MAX_FIELDS || n_out < 0) return BF_ERR_ARG;
    if (n_fields == 0 || n_out == 0) return BF_OK;
    RowsArgs args;
    long long most = 0;
    for (int k = 0; k < n_fields; ++k) {
        const bf_rows_field& F = fields[k];
        if (F.row_bytes <= 0 || (F.row_bytes & (F.pad == 1 ? 7 : 3)) || (F.pad != 0 && F.pad != 1) ||
            !F.dst || F.n_a < 0 || F.n_b < 0 ||
            (F.n_a > 0 && !F.a) || (F.n_b > 0 && !F.b))
            return BF_ERR_ARG;
        if (!idx && (long long)n_out != F.n_a + F.n_b) return BF_ERR_ARG;
        args.f[k] = F;
        const long long words = (long long)n_out * (F.row_bytes >> (F.pad == 1 ? 3 : 2));
        most = words > most ? words : most;
    }
    const unsigned bx = (unsigned)((most + 255) / 256 < 1024 ? (most + 255) / 256 : 1024);
    hipLaunchKernelGGL(k_rows_gather, dim3(bx, (unsigned)n_fields), dim3(256), 0, bf_stream(stream),
                       args, idx, idx_i32, n_out, status);
    return bf_check_launch();
}

// ------------------------------------------------------------------------------------------
// placement probe: where the workgroups of a launch on `stream` run.  out[2 b] = the HW_ID
// register (CU in bits 11:8, SH 12, SE 15:13), out[2 b + 1] = the XCC id; each workgroup spins
// `spin` cycles so the launch spreads over every CU the stream may use.  Checks CU-mask layouts
// (bench.py's fusion reservation) on the hardware.
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_cu_probe(int* __restrict__ out, int spin) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const long long t0 = clock64();
    while (clock64() - t0 < spin) {}
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = (int)hw;
        out[2 * blockIdx.x + 1] = (int)xcc;
    }
}

BF_API int bf_cu_probe(int* out, int n_wg, int spin, void* stream) {
    if (!out || n_wg <= 0 || spin < 0) return BF_ERR_ARG;
    hipLaunchKernelGGL(k_cu_probe, dim3(n_wg), dim3(64), 0, bf_stream(stream), out, spin);
    return bf_check_launch();
}
