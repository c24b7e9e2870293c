// Probe: store throughput by row-segment shape per wave-instruction (16 B per lane, dwordx4 stores):
// SEG bytes contiguous per row, 1024 / SEG rows per instruction; every CU streams its own region of a
// bf16-sized output matrix (row pitch PITCH bytes) the way a GEMM epilogue sweeps its tile.
#include <hip/hip_runtime.h>
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int SEG>
__global__ void __launch_bounds__(512) k_store(unsigned char* out, long long pitch, int rows_per_block,
                                               int cols_bytes) {
    constexpr int LPR = SEG / 16;          // lanes per row segment
    constexpr int RPI = 64 / LPR;          // rows per wave-instruction
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r_in = lane / LPR, c_in = (lane % LPR) * 16;
    const long long row0 = (long long)blockIdx.x * rows_per_block;
    const u32x4 v = (u32x4){(unsigned)lane, 1u, 2u, 3u};
    // each wave takes column slabs of SEG bytes, sweeps the block's rows RPI at a time
    for (int cs = wave * SEG; cs < cols_bytes; cs += 8 * SEG)
        for (int r = 0; r < rows_per_block; r += RPI)
            *reinterpret_cast<u32x4*>(out + (row0 + r + r_in) * pitch + cs + c_in) = v;
}

extern "C" int store_launch(int seg, void* out, long long pitch, int blocks, int rows_per_block, int cols_bytes,
                            void* stream) {
    hipStream_t st = (hipStream_t)stream;
    switch (seg) {
    case 32: hipLaunchKernelGGL((k_store<32>), dim3(blocks), dim3(512), 0, st, (unsigned char*)out, pitch, rows_per_block, cols_bytes); break;
    case 64: hipLaunchKernelGGL((k_store<64>), dim3(blocks), dim3(512), 0, st, (unsigned char*)out, pitch, rows_per_block, cols_bytes); break;
    case 128: hipLaunchKernelGGL((k_store<128>), dim3(blocks), dim3(512), 0, st, (unsigned char*)out, pitch, rows_per_block, cols_bytes); break;
    case 256: hipLaunchKernelGGL((k_store<256>), dim3(blocks), dim3(512), 0, st, (unsigned char*)out, pitch, rows_per_block, cols_bytes); break;
    case 512: hipLaunchKernelGGL((k_store<512>), dim3(blocks), dim3(512), 0, st, (unsigned char*)out, pitch, rows_per_block, cols_bytes); break;
    default: return -1;
    }
    return (int)hipGetLastError();
}
