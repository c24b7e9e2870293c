// bf_gemm_tune.hip — per-shape choice between the hand-written GEMM (bf_gemm.hip) and hipBLASLt
// for the plain linears of the path: bf16 A [M,K] x W [N,K]^T + bias, written bf16 or f32, or
// added to an f32 residual (D = A W^T + bias + R, hipBLASLt's beta = 1 with C = R).
//
// The first call of a shape (outside graph capture) times the hand-written kernel and every
// hipBLASLt heuristic candidate that needs no workspace (two detect streams run the same shapes
// concurrently, so a shared workspace would race) on the caller's stream, into a scratch output
// (the caller's buffers are read, never written, while timing), and keeps the fastest.  Calls
// during capture use the stored choice or the hand-written kernel.  BF_GEMM_TUNE=0: hand-written
// kernel only.  Fused GELU, row maps, residual moduli and fp8 stay on the hand-written kernels.
#include "bf_common.h"

#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

int bf_gemm_bf16_own(const void* A, int lda, const void* W, int ldw, const float* bias, const float* resid,
                     int ldr, int resid_mod, void* C, int ldc, int c_bf16, const int32_t* row_map, int M, int N,
                     int K, int act, void* stream);
int bf_gemm_fp8_own(const void* A, int lda, const void* W, int ldw, float scale, const float* bias,
                    const float* resid, int ldr, void* C, int ldc, int out_kind, float out_qscale, int M, int N,
                    int K, int act, void* stream);

namespace {

struct Plan {
    int choice = -1;                    // -1: hand-written kernel, else hipBLASLt
    hipblasLtMatmulDesc_t desc = nullptr;
    hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr, ld = nullptr;
    hipblasLtMatmulAlgo_t algo;
    float us_own = 0.f, us_lib = 0.f;
};

// M, N, K, lda, ldw, ldc, ldr (-1: no residual), output bf16, bias, resid aliases C, f32 operands, act
using Key = std::tuple<int, int, int, int, int, int, int, int, int, int, int, int>;

std::mutex g_mu;
std::map<Key, Plan> g_plans;
hipblasLtHandle_t g_handle = nullptr;
int g_tune = -1;

bool tune_enabled() {
    if (g_tune < 0) {
        const char* e = getenv("BF_GEMM_TUNE");
        g_tune = e ? atoi(e) != 0 : 1;
    }
    return g_tune != 0;
}

struct Args {
    const void *A, *W;
    const float *bias, *resid;
    void* C;
    int lda, ldw, ldr, ldc, c_bf16, M, N, K;
    int f32 = 0;        // operands: 0 bf16, 2 fp8 e4m3 (bf_gemm_fp8)
    int act = 0;        // 0 (the only form handed to the library)
    float alpha = 1.f;  // fp8: the per-tensor scale product
};

hipblasStatus_t lib_call(const Plan& p, const Args& a, void* D, hipStream_t st) {
    const float alpha = a.alpha, beta = a.resid ? 1.f : 0.f;
    const void* Cin = a.resid ? static_cast<const void*>(a.resid) : D;
    return hipblasLtMatmul(g_handle, p.desc, &alpha, a.W, p.la, a.A, p.lb, &beta, Cin, p.lc, D, p.ld, &p.algo,
                           nullptr, 0, st);
}

// mean time of `reps` calls after one warm-up call, µs
template <class F>
float time_us(F&& f, hipStream_t st, int reps) {
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess) return 1e30f;
    if (hipEventCreate(&e1) != hipSuccess) { hipEventDestroy(e0); return 1e30f; }
    bool ok = f();
    (void)hipEventRecord(e0, st);
    for (int i = 0; i < reps && ok; ++i) ok = f();
    (void)hipEventRecord(e1, st);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return ok ? 1e3f * ms / reps : 1e30f;
}

void make_plan(Plan& p, const Args& a, hipStream_t st) {
    if (!g_handle && hipblasLtCreate(&g_handle) != HIPBLAS_STATUS_SUCCESS) {
        g_handle = nullptr;
        return;
    }
    // column-major view: D^T [N, M] = W [N, K] . A^T [K, M]
    if (hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return;
    const hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof ta);
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof tb);
    const uint32_t epi = a.bias ? HIPBLASLT_EPILOGUE_BIAS : HIPBLASLT_EPILOGUE_DEFAULT;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof epi);
    if (a.bias) {
        const hipDataType bt = HIP_R_32F;
        hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof bt);
        // the pointer is set per call (bias_ptr); any valid one for the heuristic query
        hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &a.bias, sizeof a.bias);
    }
    const hipDataType dt = a.c_bf16 ? HIP_R_16BF : HIP_R_32F;
    const hipDataType ot = a.f32 == 2 ? HIP_R_8F_E4M3 : HIP_R_16BF;
    hipblasLtMatrixLayoutCreate(&p.la, ot, a.K, a.N, a.ldw);
    hipblasLtMatrixLayoutCreate(&p.lb, ot, a.K, a.M, a.lda);
    hipblasLtMatrixLayoutCreate(&p.lc, dt, a.N, a.M, a.resid ? a.ldr : a.ldc);
    hipblasLtMatrixLayoutCreate(&p.ld, dt, a.N, a.M, a.ldc);
    hipblasLtMatmulPreference_t pref;
    if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) return;
    const uint64_t no_ws = 0;
    hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &no_ws, sizeof no_ws);
    hipblasLtMatmulHeuristicResult_t res[16];
    int nres = 0;
    if (hipblasLtMatmulAlgoGetHeuristic(g_handle, p.desc, p.la, p.lb, p.lc, p.ld, pref, 16, res, &nres) !=
        HIPBLAS_STATUS_SUCCESS)
        nres = 0;
    hipblasLtMatmulPreferenceDestroy(pref);
    // scratch output: the caller's C is only read (as the residual) while the candidates run
    void* D = nullptr;
    const size_t dbytes = (size_t)a.M * a.ldc * (a.c_bf16 ? 2 : 4);
    if (hipMalloc(&D, dbytes) != hipSuccess) { (void)hipGetLastError(); return; }
    const float* resid_in = a.resid;
    auto own = [&] {
        if (a.f32 == 2)
            return bf_gemm_fp8_own(a.A, a.lda, a.W, a.ldw, a.alpha, a.bias, resid_in, a.ldr, D, a.ldc,
                                   a.c_bf16 ? 1 : 0, 1.f, a.M, a.N, a.K, 0, st) == BF_OK;
        return bf_gemm_bf16_own(a.A, a.lda, a.W, a.ldw, a.bias, resid_in, a.ldr, 0, D, a.ldc, a.c_bf16, nullptr,
                                a.M, a.N, a.K, 0, st) == BF_OK;
    };
    // two passes over every candidate (own kernel first in the first, last in the second: a clock
    // still ramping up or a neighbour's burst cannot favour one side), the minimum of each kept
    std::vector<float> lib_us(nres, 1e30f);
    p.us_own = 1e30f;
    for (int pass = 0; pass < 2; ++pass) {
        if (pass == 0) p.us_own = std::min(p.us_own, time_us(own, st, 3));
        for (int r = 0; r < nres; ++r) {
            if (res[r].state != HIPBLAS_STATUS_SUCCESS || res[r].workspaceSize != 0) continue;
            Plan q = p;
            q.algo = res[r].algo;
            lib_us[r] = std::min(lib_us[r],
                                 time_us([&] { return lib_call(q, a, D, st) == HIPBLAS_STATUS_SUCCESS; }, st, 3));
        }
        if (pass == 1) p.us_own = std::min(p.us_own, time_us(own, st, 3));
    }
    // a stable choice across boxes: the library only when it wins by more than 5 %, and then its
    // first candidate (heuristic order) within 3 % of its best, so timing noise between near-equal
    // candidates does not change the kernel -- and with it the summation order -- from run to run
    p.us_lib = 1e30f;
    for (int r = 0; r < nres; ++r) p.us_lib = std::min(p.us_lib, lib_us[r]);
    if (p.us_lib < 0.95f * p.us_own) {
        for (int r = 0; r < nres; ++r)
            if (lib_us[r] <= 1.03f * p.us_lib) {
                p.choice = r;
                p.algo = res[r].algo;
                break;
            }
    }
    (void)hipStreamSynchronize(st);
    (void)hipFree(D);
    if (getenv("BF_GEMM_TUNE_LOG"))
        fprintf(stderr, "bf_gemm tune %s M=%d N=%d K=%d out=%s resid=%d bias=%d act=%d: own %.1f us, hipBLASLt best "
                "%.1f us (%d candidates) -> %s\n", a.f32 == 2 ? "fp8" : "bf16", a.M, a.N, a.K, a.c_bf16 ? "bf16" : "f32",
                a.resid != nullptr, a.bias != nullptr, a.act, p.us_own, p.us_lib, nres,
                p.choice < 0 ? "own" : "hipBLASLt");
}

}  // namespace

// 0: the hand-written kernels only; 1: per-shape choice (default; env BF_GEMM_TUNE)
BF_API void bf_gemm_set_tune(int on) {
    std::lock_guard<std::mutex> g(g_mu);
    g_tune = on ? 1 : 0;
}

// the choices made so far, one "MxNxK out resid bias: own us / hipBLASLt us -> choice" per line;
// returns the bytes needed (without the terminator)
BF_API int bf_gemm_tune_report(char* buf, int cap) {
    std::lock_guard<std::mutex> g(g_mu);
    std::string out;
    char line[200];
    for (const auto& kv : g_plans) {
        const Key& k = kv.first;
        const Plan& p = kv.second;
        snprintf(line, sizeof line, "%s %dx%dx%d %s%s%s%s: own %.1f us, hipBLASLt %.1f us -> %s\n",
                 std::get<10>(k) == 2 ? "fp8" : "bf16", std::get<0>(k), std::get<1>(k), std::get<2>(k),
                 std::get<7>(k) ? "bf16" : "f32", std::get<6>(k) >= 0 ? " +resid" : "", std::get<8>(k) ? " +bias" : "",
                 std::get<11>(k) == 2 ? " +relu" : "", p.us_own, p.us_lib < 1e29f ? p.us_lib : -1.f,
                 p.choice < 0 ? "own" : "hipBLASLt");
        out += line;
    }
    if (buf && cap > 0) {
        const int n = (int)std::min(out.size(), (size_t)cap - 1);
        memcpy(buf, out.data(), n);
        buf[n] = 0;
    }
    return (int)out.size();
}

namespace {

int tuned_call(const Args& a, void* stream) {
    if (!tune_enabled() || (a.resid && a.c_bf16) || (a.resid && a.act)) return 1;
    hipStream_t st = bf_stream(stream);
    const Key key{a.M, a.N, a.K, a.lda, a.ldw, a.ldc, a.resid ? a.ldr : -1, a.c_bf16, a.bias != nullptr,
                  a.resid == a.C ? 1 : 0, a.f32, a.act};
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_plans.find(key);
    if (it == g_plans.end()) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
            (void)hipGetLastError();
            return 1;                              // no timing inside a capture
        }
        Plan p;
        make_plan(p, a, st);
        it = g_plans.emplace(key, p).first;
    }
    Plan& p = it->second;
    if (p.choice < 0) return 1;
    if (a.bias)
        hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &a.bias, sizeof a.bias);
    return lib_call(p, a, a.C, st) == HIPBLAS_STATUS_SUCCESS ? BF_OK : BF_ERR_LAUNCH;
}

}  // namespace

// 1: not handled here (the caller runs the hand-written kernel); otherwise a bf_status
int bf_gemm_tuned(const void* A, int lda, const void* W, int ldw, const float* bias, const float* resid, int ldr,
                  void* C, int ldc, int c_bf16, int M, int N, int K, void* stream) {
    return tuned_call(Args{A, W, bias, resid, C, lda, ldw, ldr, ldc, c_bf16, M, N, K, 0, 0}, stream);
}

// the fp8 CLIP linears with a bf16 output or an f32 (residual) output and no activation
// (configs[4]); scale = the activation x weight scale product, hipBLASLt's alpha
int bf_gemm_fp8_tuned(const void* A, int lda, const void* W, int ldw, float scale, const float* bias,
                      const float* resid, int ldr, void* C, int ldc, int out_kind, int M, int N, int K, int act,
                      void* stream) {
    if (act != 0 || out_kind > 1) return 1;
    Args a{A, W, bias, resid, C, lda, ldw, ldr, ldc, out_kind == 1 ? 1 : 0, M, N, K, 2, 0};
    a.alpha = scale;
    return tuned_call(a, stream);
}

