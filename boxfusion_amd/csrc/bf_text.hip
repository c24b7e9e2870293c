// bf_text.hip — the CLIP text tower's non-GEMM steps (precompute_class_features.py:37-43, the
// open_clip "ViT-H-14" encode_text the reference's commented path calls):
//   bf_token_embed        token_embedding(ids) + positional_embedding       (f32 rows)
//   bf_text_pool          x[n, argmax(ids[n])] (the EOT token: highest id, first occurrence)
//   bf_l2_normalize_rows  x / ||x||_2 per row (precompute_class_features.py:43)
// The transformer blocks run on bf_layernorm / bf_gemm_bf16 / bf_attention_causal.
#include "bf_common.h"

#include <climits>

// one thread per 16-B chunk of an output row: ids i32 [n_tok], table f32 [vocab, W],
// pos f32 [S, W] (token t sits at position t % S)
__global__ void __launch_bounds__(256) k_token_embed(const int32_t* __restrict__ ids, int n_tok,
                                                     const float* __restrict__ table, int vocab,
                                                     const float* __restrict__ pos, int S, int W,
                                                     float* __restrict__ out, int32_t* __restrict__ status) {
    const int cpr = W / 4;
    const long long total = (long long)n_tok * cpr;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (long long)gridDim.x * blockDim.x) {
        const int t = (int)(e / cpr), c = (int)(e - (long long)t * cpr) * 4;
        const int id = ids[t];
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (id >= 0 && id < vocab) {
            v = *reinterpret_cast<const float4*>(table + (size_t)id * W + c);
        } else if (status && c == 0) {
            atomicOr(status, BF_DEV_INDEX_RANGE);
        }
        const float4 p = *reinterpret_cast<const float4*>(pos + (size_t)(t % S) * W + c);
        v.x += p.x; v.y += p.y; v.z += p.z; v.w += p.w;
        *reinterpret_cast<float4*>(out + (size_t)t * W + c) = v;
    }
}

BF_API int bf_token_embed(const int32_t* ids, int n_tok, const float* table, int vocab, const float* pos,
                          int S, int W, float* out, int32_t* status, void* stream) {
    if (!ids || !table || !pos || !out || n_tok < 0 || vocab <= 0 || S <= 0 || W <= 0 || W % 4)
        return BF_ERR_ARG;
    if (n_tok == 0) return BF_OK;
    const long long total = (long long)n_tok * (W / 4);
    const unsigned g = (unsigned)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    hipLaunchKernelGGL(k_token_embed, dim3(g), dim3(256), 0, bf_stream(stream), ids, n_tok, table, vocab,
                       pos, S, W, out, status);
    return bf_check_launch();
}

// one 256-thread workgroup per prompt: wave 0 finds the first argmax of the prompt's ids (torch
// argmax semantics), then every thread copies a slice of that row
__global__ void __launch_bounds__(256) k_text_pool(const int32_t* __restrict__ ids, int S,
                                                   const float* __restrict__ x, int W,
                                                   float* __restrict__ out) {
    __shared__ int s_pos;
    const int n = blockIdx.x, t = threadIdx.x;
    if (t < 64) {
        int best = INT_MIN, bpos = 0;
        for (int s = t; s < S; s += 64) {
            const int v = ids[(size_t)n * S + s];
            if (v > best) { best = v; bpos = s; }        // first occurrence within the lane
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const int ob = __shfl_xor(best, o, 64), op = __shfl_xor(bpos, o, 64);
            if (ob > best || (ob == best && op < bpos)) { best = ob; bpos = op; }
        }
        if (t == 0) s_pos = bpos;
    }
    __syncthreads();
    const float* src = x + ((size_t)n * S + s_pos) * W;
    for (int c = t; c < W; c += blockDim.x) out[(size_t)n * W + c] = src[c];
}

BF_API int bf_text_pool(const int32_t* ids, int N, int S, const float* x, int W, float* out, void* stream) {
    if (!ids || !x || !out || N < 0 || S <= 0 || W <= 0) return BF_ERR_ARG;
    if (N == 0) return BF_OK;
    hipLaunchKernelGGL(k_text_pool, dim3((unsigned)N), dim3(256), 0, bf_stream(stream), ids, S, x, W, out);
    return bf_check_launch();
}

// one 256-thread workgroup per row: sum of squares (f32, tree order), then x / sqrt(sum)
__global__ void __launch_bounds__(256) k_l2norm_rows(const float* x, int W, float* out) {
    __shared__ float part[4];
    const int r = blockIdx.x, t = threadIdx.x;
    const float* row = x + (size_t)r * W;
    float s = 0.f;
    for (int c = t; c < W; c += blockDim.x) s = fmaf(row[c], row[c], s);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((t & 63) == 0) part[t >> 6] = s;
    __syncthreads();
    const float nrm = sqrtf((part[0] + part[1]) + (part[2] + part[3]));
    for (int c = t; c < W; c += blockDim.x) out[(size_t)r * W + c] = row[c] / nrm;
}

BF_API int bf_l2_normalize_rows(const float* x, int rows, int W, float* out, void* stream) {
    if (!x || !out || rows < 0 || W <= 0) return BF_ERR_ARG;
    if (rows == 0) return BF_OK;
    hipLaunchKernelGGL(k_l2norm_rows, dim3((unsigned)rows), dim3(256), 0, bf_stream(stream), x, W, out);
    return bf_check_launch();
}
