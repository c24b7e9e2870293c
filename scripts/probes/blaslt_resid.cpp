// blaslt_resid.cpp (probe): hipBLASLt on the CLIP residual GEMM shapes, bf16 A / W, f32 residual
// in place (D = C = resid, beta 1) + bias epilogue, against the same GEMM without the residual.
// Build: hipcc --offload-arch=gfx950 -O2 scripts/probes/blaslt_resid.cpp -lhipblaslt -o <out>
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { auto e_ = (x); if ((int)e_ != 0) { printf("error %d at %s:%d\n", (int)e_, __FILE__, __LINE__); exit(1); } } while (0)

extern "C" int bf_gemm_bf16(const void* A, int lda, const void* W, int ldw, const float* bias,
                            const float* resid, int ldr, int resid_mod, void* C, int ldc, int c_bf16,
                            const int32_t* row_map, int M, int N, int K, int act, void* stream);

// random bf16 in [-s, s] (hash of the index), so the clock runs as on real activations
__global__ void k_fill(unsigned short* p, size_t n, float s, unsigned seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u ^ seed;
        x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
        const float f = ((x & 0xffffff) / 16777216.f * 2.f - 1.f) * s;
        p[i] = (unsigned short)(__float_as_uint(f) >> 16);
    }
}
__global__ void k_fillf(float* p, size_t n, unsigned seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u ^ seed;
        x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
        p[i] = (x & 0xffffff) / 16777216.f * 2.f - 1.f;
    }
}

static float run_own(int M, int N, int K, bool resid, bool bf16_out, int act, void* A, void* W, float* bias,
                     void* C, int iters) {
    auto go = [&] {
        return bf_gemm_bf16(A, K, W, K, bias, resid ? (float*)C : nullptr, N, 0, C, N, bf16_out ? 1 : 0,
                            nullptr, M, N, K, act, nullptr);
    };
    for (int i = 0; i < 2; ++i) CK(go());
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    for (int i = 0; i < iters; ++i) CK(go());
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= iters;
    printf("  own     M=%d N=%d K=%d resid=%d out=%s act=%d: %.1f us = %.0f TF\n", M, N, K, (int)resid,
           bf16_out ? "bf16" : "f32", act, ms * 1e3, 2.0 * M * N * K / (ms * 1e-3) / 1e12);
    return ms;
}


static float run(hipblasLtHandle_t h, int M, int N, int K, bool resid, bool bf16_out, int epi, void* ws, size_t wsz,
                 void* A, void* W, float* bias, void* C, int iters) {
    hipblasLtMatmulDesc_t desc;
    CK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
    hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof ta));
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof tb));
    uint32_t ep = (uint32_t)epi;
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof ep));
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof bias));
    hipDataType bt = HIP_R_32F;
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof bt));
    const hipDataType dt = bf16_out ? HIP_R_16BF : HIP_R_32F;
    hipblasLtMatrixLayout_t la, lb, lc, ld;
    CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, K, N, K));   // W [N][K] row-major = K x N col-major, op T
    CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, K, M, K));   // A [M][K] row-major = K x M col-major
    CK(hipblasLtMatrixLayoutCreate(&lc, dt, N, M, N));
    CK(hipblasLtMatrixLayoutCreate(&ld, dt, N, M, N));
    hipblasLtMatmulPreference_t pref;
    CK(hipblasLtMatmulPreferenceCreate(&pref));
    uint64_t w64 = wsz;
    CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &w64, sizeof w64));
    hipblasLtMatmulHeuristicResult_t res[8];
    int nres = 0;
    CK(hipblasLtMatmulAlgoGetHeuristic(h, desc, la, lb, lc, ld, pref, 8, res, &nres));
    float alpha = 1.f, beta = resid ? 1.f : 0.f;
    float best = 1e30f;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int r = 0; r < nres; ++r) {
        for (int i = 0; i < 2; ++i)
            CK(hipblasLtMatmul(h, desc, &alpha, W, la, A, lb, &beta, C, lc, C, ld, &res[r].algo, ws, wsz, 0));
        hipEventRecord(e0, 0);
        for (int i = 0; i < iters; ++i)
            CK(hipblasLtMatmul(h, desc, &alpha, W, la, A, lb, &beta, C, lc, C, ld, &res[r].algo, ws, wsz, 0));
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms / iters < best) best = ms / iters;
        printf("    algo %d: %.1f us (ws %zu)\n", r, ms / iters * 1e3, (size_t)res[r].workspaceSize);
    }
    if (getenv("PROBE_GRAPH") && nres > 0) {     // capture one call, replay it
        hipStream_t st;
        hipStreamCreate(&st);
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        CK(hipblasLtMatmul(h, desc, &alpha, W, la, A, lb, &beta, C, lc, C, ld, &res[0].algo, ws, wsz, st));
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        hipEventRecord(e0, st);
        for (int i = 0; i < iters; ++i) CK(hipGraphLaunch(ge, st));
        hipEventRecord(e1, st);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("    graph replay of algo 0: %.1f us\n", ms / iters * 1e3);
    }
    printf("  M=%d N=%d K=%d resid=%d out=%s epi=%d: %d algos, best %.1f us = %.0f TF\n", M, N, K, (int)resid,
           bf16_out ? "bf16" : "f32", epi, nres, best * 1e3, 2.0 * M * N * K / (best * 1e-3) / 1e12);
    return best;
}

int main() {
    hipblasLtHandle_t h;
    CK(hipblasLtCreate(&h));
    const int M = 32896;
    size_t wsz = 256u << 20;
    void* ws;
    CK(hipMalloc(&ws, wsz));
    void *A, *W, *C;
    float* bias;
    CK(hipMalloc(&A, (size_t)M * 5120 * 2));
    CK(hipMalloc(&W, (size_t)5120 * 5120 * 2));
    CK(hipMalloc(&C, (size_t)M * 5120 * 4));
    CK(hipMalloc(&bias, 5120 * 4));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (unsigned short*)A, (size_t)M * 5120, 1.f, 1u);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (unsigned short*)W, (size_t)5120 * 5120, 0.02f, 2u);
    hipLaunchKernelGGL(k_fillf, dim3(4096), dim3(256), 0, 0, (float*)C, (size_t)M * 5120, 3u);
    hipLaunchKernelGGL(k_fillf, dim3(64), dim3(256), 0, 0, bias, (size_t)5120, 4u);
    CK(hipDeviceSynchronize());
    struct S { const char* name; int N, K; } shapes[] = {{"clip_fc2", 1280, 5120}, {"clip_proj", 1280, 1280},
                                                       {"clip_qkv", 3840, 1280}, {"clip_fc1", 5120, 1280}};
    for (auto& s : shapes) {
        printf("%s\n", s.name);
        for (int rep = 0; rep < 1; ++rep) {
            run_own(M, s.N, s.K, true, false, 0, A, W, bias, C, 10);
            run(h, M, s.N, s.K, true, false, HIPBLASLT_EPILOGUE_BIAS, ws, wsz, A, W, bias, C, 10);
            run_own(M, s.N, s.K, false, true, 0, A, W, bias, C, 10);
            run(h, M, s.N, s.K, false, true, HIPBLASLT_EPILOGUE_BIAS, ws, wsz, A, W, bias, C, 10);
            if (s.N == 5120) {
                run_own(M, s.N, s.K, false, true, 1, A, W, bias, C, 10);
                run(h, M, s.N, s.K, false, true, HIPBLASLT_EPILOGUE_GELU_BIAS, ws, wsz, A, W, bias, C, 10);
            }
        }
    }
    return 0;
}
