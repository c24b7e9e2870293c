// bf_depth.hip — per-frame depth work over the whole chip: trimmed depth standardisation
// (Preprocessor.standardize_depth_map, preprocessor.py:97-129) and the back-projection of the
// same depth map (tools/utils.py:232-287, demo.py:121-127), for a batch of b frames.
//
//   valid = d > 0 (NaN and <= 0 are invalid), m = #valid,
//   slice = sorted(valid)[int(0.1 m) : int(0.9 m)], mean / unbiased var of the slice,
//   std = sqrt(var + 1e-2), out = ((valid ? d : mean) - mean) / std, params = (mean, std);
//   fewer than two values in the slice: mean 0, std 1.
//
// The two order statistics (ranks klo and khi-1) come from a 3-level radix select over the
// bit patterns of the positive floats (monotone as unsigned): 11 + 10 + 10 bits.  Every level is
// one pass over the frames split into slices of CHUNK elements (one 512-thread workgroup each:
// 8192 elements for small batches, 32768 for large ones, so the grid is >= ~300 workgroups and
// each thread keeps 4-16 float4 loads in flight): LDS histogram of the level's digit among the
// elements still matching the prefix found so far, flushed to the frame's global histogram
// with one atomic per non-empty bin; the frame's last-arriving workgroup of the pass (a per-frame
// arrival counter) then locates both ranks, so no separate select launch runs between passes.  The sums the trimmed moments need ride on the same passes, on conditions known when
// the pass starts: with T a threshold bit pattern (the lower and the upper order statistic),
//   sum_{u < T} x = sum_{digit1 < t1} x               (level-2 pass, registers)
//                 + sum_{digit1 == t1, digit2 < t2} x (level-3 pass, registers)
//                 + sum_{d3 < t3} count3[d3] * value  (last select, exact products),
// and the slice sum is [sum_{u<Thi} + (khi - #{u<Thi}) vhi] - [sum_{u<Tlo} + (klo - #{u<Tlo}) vlo]
// (ties at either order statistic included exactly).  Partial sums go to per-slice slots reduced
// in a fixed order: the result does not depend on scheduling.  In double the sums of x are exact
// for depth-like data (f32 values in a 53-bit mantissa), so params and outputs equal the round-2
// single-workgroup kernel's bit for bit (scripts/depth_std_bench.py A/B).
//
// HBM passes: level 1, level 2, level 3 (reads), normalise (read + write); the selects touch only
// the histograms (four launches for small batches, seven -- the selects on their own -- for large).  Slices map to the same XCD in every pass (same grid, block id mod
// 8), so at small batches the later passes read the frames from that XCD's L2.  The normalise
// pass optionally back-projects the same pixels (bf_depth_preprocess), saving the separate
// read of bf_backproject.
#include "bf_common.h"

#define DS_T 512                   // threads per slice workgroup
#define DS_MIN_CHUNK 8192          // 4 float4 per thread
#define DS_SH1 20                  // level-1 digit: bits 30..20 (11 bits)
#define DS_SH2 10                  // level-2 digit: bits 19..10 (10 bits); level 3: bits 9..0
#define DS_NB1 2048
#define DS_NB2 1024
#define DS_NB3 1024
#define DS_SEL_T 1024              // LDS scratch sizing of the selects (they run with DS_T threads)
#ifndef DS_NORM_KV
#define DS_NORM_KV 1               // float4 groups per thread of the small-batch normalise pass
#endif

struct DsSel {
    long long m, klo, khi;
    long long below[2];   // #valid with u < the current bin's lower edge (per threshold)
    long long rank[2];    // remaining rank inside the current bin
    unsigned prefix[2];   // threshold bits found so far
    int degenerate;       // slice of fewer than 2 values: mean 0, std 1
    int pad_;
    double A[2], Q[2];    // sum x, sum x^2 over u < (current prefix's bin start)
};

struct DsLayout {
    size_t hist1, hist2, hist3, sel, part, stride;
};

__host__ __device__ inline int ds_slices(long long n, int chunk) { return (int)((n + chunk - 1) / chunk); }

__host__ __device__ inline DsLayout ds_layout(long long n) {
    DsLayout L;
    L.hist1 = 0;
    L.hist2 = L.hist1 + DS_NB1 * sizeof(unsigned);
    L.hist3 = L.hist2 + 2 * DS_NB2 * sizeof(unsigned);
    L.sel = L.hist3 + 2 * DS_NB3 * sizeof(unsigned);
    L.part = L.sel + 256;
    L.stride = L.part + (size_t)ds_slices(n, DS_MIN_CHUNK) * 8 * sizeof(double);
    L.stride = (L.stride + 255) & ~(size_t)255;
    return L;
}

__device__ __forceinline__ bool ds_valid(float x) { return x > 0.0f; }

// this thread's KV float4 groups of slice s: group it holds elements
// s*CHUNK + it*(4*DS_T) + 4*tid + {0..3} (coalesced); out-of-range elements read as 0 (invalid)
template <int KV>
__device__ __forceinline__ void ds_load(const float* __restrict__ d, long long n, int s, float4 (&v)[KV]) {
    constexpr int CHUNK = KV * 4 * DS_T;
    const long long base = (long long)s * CHUNK;
    if ((n & 3) == 0 && ((reinterpret_cast<uintptr_t>(d) & 15) == 0)) {
        // float4 groups; a group past the end (only in a frame's last slice) reads as invalid
#pragma unroll
        for (int it = 0; it < KV; ++it) {
            const long long i0 = base + (long long)it * 4 * DS_T + 4 * threadIdx.x;
            v[it] = i0 < n ? *reinterpret_cast<const float4*>(d + i0) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    } else {
#pragma unroll
        for (int it = 0; it < KV; ++it) {
            const long long i0 = base + (long long)it * 4 * DS_T + 4 * threadIdx.x;
            v[it].x = i0 < n ? d[i0] : 0.0f;
            v[it].y = i0 + 1 < n ? d[i0 + 1] : 0.0f;
            v[it].z = i0 + 2 < n ? d[i0 + 2] : 0.0f;
            v[it].w = i0 + 3 < n ? d[i0 + 3] : 0.0f;
        }
    }
}

template <int KV, typename F>
__device__ __forceinline__ void ds_each(const float4 (&v)[KV], F&& f) {
#pragma unroll
    for (int it = 0; it < KV; ++it) {
        f(v[it].x); f(v[it].y); f(v[it].z); f(v[it].w);
    }
}

// flush a workgroup's LDS histogram to the frame's global one (atomics on non-empty bins only)
__device__ __forceinline__ void ds_flush(const unsigned* h, unsigned* g, int nb) {
    for (int b = threadIdx.x; b < nb; b += blockDim.x) {
        const unsigned c = h[b];
        if (c) atomicAdd(g + b, c);
    }
}

// workgroup sum of 4 doubles (fixed order: wave butterfly, then the waves in order; thread 0)
__device__ __forceinline__ void ds_block_sum4(double (&v)[4], double (*scratch)[16]) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
        for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o, 64);
    if (bf_lane() == 0)
#pragma unroll
        for (int k = 0; k < 4; ++k) scratch[k][threadIdx.x >> 6] = v[k];
    __syncthreads();
    if (threadIdx.x == 0)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            double s = 0.0;
            for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += scratch[k][i];
            v[k] = s;
        }
}

// locate rank r of histogram h[NB] (LDS) in a block scan: thread t owns bins [t*per, (t+1)*per).
// Writes (bin, count below) to res (LDS) for the thread that holds it; r < 0 skips.
// Returns the histogram total (every thread).
template <int NB>
__device__ long long ds_scan_locate(const unsigned* h, long long r0, long long r1, long long (*res)[2],
                                    long long* s_w) {
    const int T = blockDim.x, t = threadIdx.x, per = NB / T;
    long long own = 0;
    for (int k = 0; k < per; ++k) own += h[t * per + k];
    long long incl = own;
    for (int o = 1; o < 64; o <<= 1) {
        const long long y = __shfl_up(incl, o, 64);
        if (bf_lane() >= o) incl += y;
    }
    if (bf_lane() == 63) s_w[t >> 6] = incl;
    __syncthreads();
    long long off = 0, total = 0;
    for (int w = 0; w < T / 64; ++w) {
        if (w < (t >> 6)) off += s_w[w];
        total += s_w[w];
    }
    const long long excl = off + incl - own;
    const long long rr[2] = {r0, r1};
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const long long r = rr[q];
        if (r >= excl && r < excl + own) {
            long long c = excl;
            for (int k = 0; k < per; ++k) {
                const long long hb = h[t * per + k];
                if (r < c + hb) { res[q][0] = t * per + k; res[q][1] = c; break; }
                c += hb;
            }
        }
    }
    __syncthreads();
    return total;
}

// take nb global bins into LDS and clear them for the next call.  The bins were filled by other
// workgroups of the same launch (on every XCD): device-coherent loads (agent-scope atomics) read
// them where those atomics landed, not a stale line of this XCD's L2; all of a thread's loads are
// in flight at once (nb / blockDim <= 4), then the bins are cleared the same way.
__device__ __forceinline__ void ds_take(unsigned* __restrict__ g, unsigned* __restrict__ h, int nb) {
    unsigned v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int b = threadIdx.x + k * blockDim.x;
        v[k] = b < nb ? __hip_atomic_load(g + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int b = threadIdx.x + k * blockDim.x;
        if (b < nb) {
            h[b] = v[k];
            __hip_atomic_store(g + b, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// device-coherent 64-bit store / load of the per-slice partial sums (written by the slice
// workgroups, read by the frame's last-arriving one in the same launch)
__device__ __forceinline__ void ds_put(double* p, double v) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ds_get(const double* p) {
    return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<const unsigned long long*>(p),
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// fixed-order sum of per-slice partials p[s*8 + o + k], k < 4 (one slice per thread, a wave
// butterfly, the waves in order): every thread gets the result
__device__ void ds_reduce_partials(const double* __restrict__ p, int ns, int o, double (&a)[4],
                                   double (*s_p)[DS_SEL_T / 64]) {
    double v[4] = {0.0, 0.0, 0.0, 0.0};
    for (int i = threadIdx.x; i < ns; i += blockDim.x)
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] += ds_get(p + (size_t)i * 8 + o + k);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        for (int s = 32; s > 0; s >>= 1) v[k] += __shfl_xor(v[k], s, 64);
    if (bf_lane() == 0)
#pragma unroll
        for (int k = 0; k < 4; ++k) s_p[k][threadIdx.x >> 6] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        double t = 0.0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += s_p[k][w];
        a[k] = t;
    }
}

// select after level 1 (run by the frame's last-arriving level-1 workgroup): m, klo, khi and both
// thresholds' level-1 bins; clears hist1
__device__ __forceinline__ void ds_sel1(int f, long long n, unsigned char* __restrict__ ws, unsigned* h) {
    __shared__ long long s_w[DS_SEL_T / 64], s_res[2][2];
    const DsLayout L = ds_layout(n);
    unsigned char* base = ws + (size_t)f * L.stride;
    DsSel* S = reinterpret_cast<DsSel*>(base + L.sel);
    ds_take(reinterpret_cast<unsigned*>(base + L.hist1), h, DS_NB1);
    if (threadIdx.x < 2) { s_res[threadIdx.x][0] = 0; s_res[threadIdx.x][1] = 0; }
    __syncthreads();
    // the ranks depend on the total: one scan for the count, one to locate both ranks
    const long long m = ds_scan_locate<DS_NB1>(h, -1, -1, s_res, s_w);
    const long long klo = (long long)(0.1 * (double)m);
    const long long khi = (long long)((1.0 - 0.1) * (double)m);
    const int degenerate = (khi - klo) <= 1;
    if (!degenerate) ds_scan_locate<DS_NB1>(h, klo, khi - 1, s_res, s_w);
    if (threadIdx.x == 0) {
        S->m = m; S->klo = klo; S->khi = khi;
        S->degenerate = degenerate;
        const long long rk[2] = {klo, khi - 1};
        for (int q = 0; q < 2; ++q) {
            S->prefix[q] = (unsigned)s_res[q][0] << DS_SH1;
            S->below[q] = s_res[q][1];
            S->rank[q] = degenerate ? 0 : rk[q] - s_res[q][1];
            S->A[q] = 0.0; S->Q[q] = 0.0;
        }
    }
}


// Per-frame arrival of a slice workgroup at the end of a pass (counter `c` of the frame's select
// block).  Everything the slices share inside a launch goes through device-coherent atomics (the
// histogram adds, ds_put / ds_get, ds_take's exchanges), so no cache-wide fence is needed (an
// agent-scope fence writes back the XCD's whole L2: 3x slower measured): every thread waits for
// its own atomics to complete, the workgroup barrier orders them before thread 0's arrival, and
// the LAST workgroup of the frame (the only one to return true) runs the frame's select in place
// of a separate one-workgroup-per-frame launch.  It resets the counter: the workspace is left as
// it was found.
#define DS_ARRIVE 192   // byte offset of the three pass counters inside the 256-B select block
__device__ __forceinline__ bool ds_last_arrival(unsigned char* sel_arrive, int c, int total) {
    __shared__ int s_last;
    unsigned* ctr = reinterpret_cast<unsigned*>(sel_arrive) + c;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned old = atomicAdd(ctr, 1u);
        s_last = old == (unsigned)(total - 1);
        if (s_last) atomicExch(ctr, 0u);
    }
    __syncthreads();
    return s_last != 0;
}

// ------------------------------------------------------------------------------------------
// level 1: 11-bit digit histogram of every valid value; the frame's last workgroup selects
// ------------------------------------------------------------------------------------------
template <int KV, bool FSEL>
__global__ void __launch_bounds__(DS_T) k_ds_hist1(const float* __restrict__ depth, long long n,
                                                   unsigned char* __restrict__ ws) {
    __shared__ __align__(16) unsigned h[DS_NB1];
    const int s = blockIdx.x, f = blockIdx.y;
    float4 v[KV];
    ds_load<KV>(depth + (size_t)f * n, n, s, v);          // loads in flight while LDS clears
    const DsLayout L = ds_layout(n);
    unsigned* g = reinterpret_cast<unsigned*>(ws + (size_t)f * L.stride + L.hist1);
    for (int b = threadIdx.x * 4; b < DS_NB1; b += DS_T * 4)
        *reinterpret_cast<uint4*>(h + b) = make_uint4(0, 0, 0, 0);
    __syncthreads();
    ds_each<KV>(v, [&](float x) {
        if (ds_valid(x)) atomicAdd(h + (__float_as_uint(x) >> DS_SH1), 1u);
    });
    __syncthreads();
    ds_flush(h, g, DS_NB1);
    if (FSEL && ds_last_arrival(ws + (size_t)f * L.stride + L.sel + DS_ARRIVE, 0, gridDim.x)) ds_sel1(f, n, ws, h);
}

// ------------------------------------------------------------------------------------------
// level 2: sums below each threshold's level-1 bin + level-2 digit histograms inside the bins
// ------------------------------------------------------------------------------------------

__device__ __forceinline__ void ds_sel2(int f, long long n, int chunk, unsigned char* __restrict__ ws,
                                        unsigned (&h)[2][DS_NB2]);
__device__ __forceinline__ void ds_fin(int f, long long n, int chunk, unsigned char* __restrict__ ws,
                                       float* __restrict__ params, unsigned (&h)[2][DS_NB3]);

template <int KV, bool FSEL>
__global__ void __launch_bounds__(DS_T) k_ds_hist2(const float* __restrict__ depth, long long n,
                                                   unsigned char* __restrict__ ws) {
    constexpr int CHUNK = KV * 4 * DS_T;
    __shared__ __align__(16) unsigned h[2][DS_NB2];
    __shared__ double scratch[4][16];
    const int s = blockIdx.x, f = blockIdx.y;
    float4 v[KV];
    ds_load<KV>(depth + (size_t)f * n, n, s, v);
    const DsLayout L = ds_layout(n);
    unsigned char* base = ws + (size_t)f * L.stride;
    const DsSel* S = reinterpret_cast<const DsSel*>(base + L.sel);
    const int degenerate = S->degenerate;
    const unsigned b0 = S->prefix[0] >> DS_SH1, b1 = S->prefix[1] >> DS_SH1;
    if (!degenerate) {                                   // (workgroup-uniform)
        for (int b = threadIdx.x * 4; b < 2 * DS_NB2; b += DS_T * 4)
            *reinterpret_cast<uint4*>(&h[0][0] + b) = make_uint4(0, 0, 0, 0);
        __syncthreads();
        double a[4] = {0.0, 0.0, 0.0, 0.0};   // A0, Q0, A1, Q1
        ds_each<KV>(v, [&](float x) {
            if (!ds_valid(x)) return;
            const unsigned u = __float_as_uint(x), k1 = u >> DS_SH1, k2 = (u >> DS_SH2) & (DS_NB2 - 1);
            const double xd = (double)x;
            if (k1 < b0) { a[0] += xd; a[1] += xd * xd; }
            if (k1 < b1) { a[2] += xd; a[3] += xd * xd; }
            if (k1 == b0) atomicAdd(&h[0][k2], 1u);
            if (k1 == b1) atomicAdd(&h[1][k2], 1u);
        });
        ds_block_sum4(a, scratch);
        __syncthreads();
        ds_flush(&h[0][0], reinterpret_cast<unsigned*>(base + L.hist2), 2 * DS_NB2);
        if (threadIdx.x == 0) {
            double* p = reinterpret_cast<double*>(base + L.part) + (size_t)s * 8;
            ds_put(p + 0, a[0]); ds_put(p + 1, a[1]); ds_put(p + 2, a[2]); ds_put(p + 3, a[3]);
        }
    }
    if (FSEL && ds_last_arrival(base + L.sel + DS_ARRIVE, 1, gridDim.x)) ds_sel2(f, n, CHUNK, ws, h);
}

// select after level 2 (the frame's last level-2 workgroup)
__device__ __forceinline__ void ds_sel2(int f, long long n, int chunk, unsigned char* __restrict__ ws,
                                        unsigned (&h)[2][DS_NB2]) {
    __shared__ long long s_w[DS_SEL_T / 64], s_res[2][2];
    __shared__ double s_p[4][DS_SEL_T / 64];
    const DsLayout L = ds_layout(n);
    unsigned char* base = ws + (size_t)f * L.stride;
    DsSel* S = reinterpret_cast<DsSel*>(base + L.sel);
    // every global read issued up front (one latency): the selection state, the histograms
    // (cleared on the way: all zero for a degenerate frame) and the per-slice partial sums
    const DsSel S0 = *S;
    ds_take(reinterpret_cast<unsigned*>(base + L.hist2), &h[0][0], 2 * DS_NB2);
    double a[4];
    ds_reduce_partials(reinterpret_cast<const double*>(base + L.part), ds_slices(n, chunk), 0, a, s_p);
    if (S0.degenerate) return;
    const long long r0 = S0.rank[0], r1 = S0.rank[1];
    if (threadIdx.x < 2) { s_res[threadIdx.x][0] = 0; s_res[threadIdx.x][1] = 0; }
    __syncthreads();
    long long bins[2], bel[2];
    ds_scan_locate<DS_NB2>(h[0], r0, -1, s_res, s_w);
    bins[0] = s_res[0][0]; bel[0] = s_res[0][1];
    __syncthreads();
    ds_scan_locate<DS_NB2>(h[1], -1, r1, s_res, s_w);
    bins[1] = s_res[1][0]; bel[1] = s_res[1][1];
    if (threadIdx.x == 0)
        for (int q = 0; q < 2; ++q) {
            S->A[q] = a[2 * q];
            S->Q[q] = a[2 * q + 1];
            S->prefix[q] = S0.prefix[q] | ((unsigned)bins[q] << DS_SH2);
            S->below[q] = S0.below[q] + bel[q];
            S->rank[q] = S0.rank[q] - bel[q];
        }
}

// ------------------------------------------------------------------------------------------
// level 3: sums inside the level-1 bin below the level-2 digit + the last histograms
// ------------------------------------------------------------------------------------------
template <int KV, bool FSEL>
__global__ void __launch_bounds__(DS_T) k_ds_hist3(const float* __restrict__ depth, long long n,
                                                   unsigned char* __restrict__ ws, float* __restrict__ params) {
    constexpr int CHUNK = KV * 4 * DS_T;
    __shared__ __align__(16) unsigned h[2][DS_NB3];
    __shared__ double scratch[4][16];
    const int s = blockIdx.x, f = blockIdx.y;
    float4 v[KV];
    ds_load<KV>(depth + (size_t)f * n, n, s, v);
    const DsLayout L = ds_layout(n);
    unsigned char* base = ws + (size_t)f * L.stride;
    const DsSel* S = reinterpret_cast<const DsSel*>(base + L.sel);
    const int degenerate = S->degenerate;
    const unsigned p0 = S->prefix[0] >> DS_SH2, p1 = S->prefix[1] >> DS_SH2;   // 21-bit prefixes
    if (!degenerate) {                                   // (workgroup-uniform)
        for (int b = threadIdx.x * 4; b < 2 * DS_NB3; b += DS_T * 4)
            *reinterpret_cast<uint4*>(&h[0][0] + b) = make_uint4(0, 0, 0, 0);
        __syncthreads();
        constexpr int D2 = DS_SH1 - DS_SH2;
        double a[4] = {0.0, 0.0, 0.0, 0.0};
        ds_each<KV>(v, [&](float x) {
            if (!ds_valid(x)) return;
            const unsigned u = __float_as_uint(x), p = u >> DS_SH2;
            const double xd = (double)x;
            // same level-1 bin, lower level-2 digit
            if ((p >> D2) == (p0 >> D2) && p < p0) { a[0] += xd; a[1] += xd * xd; }
            if ((p >> D2) == (p1 >> D2) && p < p1) { a[2] += xd; a[3] += xd * xd; }
            if (p == p0) atomicAdd(&h[0][u & (DS_NB3 - 1)], 1u);
            if (p == p1) atomicAdd(&h[1][u & (DS_NB3 - 1)], 1u);
        });
        ds_block_sum4(a, scratch);
        __syncthreads();
        ds_flush(&h[0][0], reinterpret_cast<unsigned*>(base + L.hist3), 2 * DS_NB3);
        if (threadIdx.x == 0) {
            double* p = reinterpret_cast<double*>(base + L.part) + (size_t)s * 8 + 4;
            ds_put(p + 0, a[0]); ds_put(p + 1, a[1]); ds_put(p + 2, a[2]); ds_put(p + 3, a[3]);
        }
    }
    if (FSEL && ds_last_arrival(base + L.sel + DS_ARRIVE, 2, gridDim.x)) ds_fin(f, n, CHUNK, ws, params, h);
}

// last select: the exact order statistics, the trimmed moments, params
__device__ __forceinline__ void ds_fin(int f, long long n, int chunk, unsigned char* __restrict__ ws,
                                       float* __restrict__ params, unsigned (&h)[2][DS_NB3]) {
    __shared__ long long s_w[DS_SEL_T / 64], s_res[2][2];
    __shared__ double s_p[4][DS_SEL_T / 64];
    __shared__ double s_c[4][DS_SEL_T / 64];
    const DsLayout L = ds_layout(n);
    unsigned char* base = ws + (size_t)f * L.stride;
    const DsSel S0 = *reinterpret_cast<const DsSel*>(base + L.sel);
    const int t = threadIdx.x;
    ds_take(reinterpret_cast<unsigned*>(base + L.hist3), &h[0][0], 2 * DS_NB3);
    double a[4];
    ds_reduce_partials(reinterpret_cast<const double*>(base + L.part), ds_slices(n, chunk), 4, a, s_p);
    if (S0.degenerate) {
        if (t == 0) { params[2 * f] = 0.0f; params[2 * f + 1] = 1.0f; }
        return;
    }
    const long long r0 = S0.rank[0], r1 = S0.rank[1];
    const unsigned pre0 = S0.prefix[0], pre1 = S0.prefix[1];
    if (t < 2) { s_res[t][0] = 0; s_res[t][1] = 0; }
    __syncthreads();
    long long bins[2], bel[2];
    ds_scan_locate<DS_NB3>(h[0], r0, -1, s_res, s_w);
    bins[0] = s_res[0][0]; bel[0] = s_res[0][1];
    __syncthreads();
    ds_scan_locate<DS_NB3>(h[1], -1, r1, s_res, s_w);
    bins[1] = s_res[1][0]; bel[1] = s_res[1][1];
    // exact sums of the values below each threshold inside its 21-bit prefix: bin k is the
    // single value prefix | k (one bin per thread, fixed-order reduction)
    const unsigned pre[2] = {pre0, pre1};
    double c[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < 2; ++q)
        for (int k = t; k < (int)bins[q]; k += blockDim.x) {
            const unsigned cnt = h[q][k];
            const double x = (double)__uint_as_float(pre[q] | (unsigned)k);
            c[2 * q] += (double)cnt * x;
            c[2 * q + 1] += (double)cnt * (x * x);
        }
#pragma unroll
    for (int k = 0; k < 4; ++k)
        for (int o = 32; o > 0; o >>= 1) c[k] += __shfl_xor(c[k], o, 64);
    if (bf_lane() == 0)
#pragma unroll
        for (int k = 0; k < 4; ++k) s_c[k][t >> 6] = c[k];
    __syncthreads();
    if (t == 0) {
        double cs[4] = {0.0, 0.0, 0.0, 0.0};
        for (int k = 0; k < 4; ++k)
            for (int w = 0; w < (int)(blockDim.x >> 6); ++w) cs[k] += s_c[k][w];
        double sum_below[2], sq_below[2], val[2];
        long long cnt_below[2];
        for (int q = 0; q < 2; ++q) {
            val[q] = (double)__uint_as_float(pre[q] | (unsigned)bins[q]);
            cnt_below[q] = S0.below[q] + bel[q];
            sum_below[q] = S0.A[q] + a[2 * q] + cs[2 * q];
            sq_below[q] = S0.Q[q] + a[2 * q + 1] + cs[2 * q + 1];
        }
        const long long klo = S0.klo, khi = S0.khi, Ls = khi - klo;
        // sum over sorted ranks [0, k) = sum_{u < T} + (k - #{u < T}) * v(T)
        const double nh = (double)(khi - cnt_below[1]), nl = (double)(klo - cnt_below[0]);
        const double Ssum = (sum_below[1] + nh * val[1]) - (sum_below[0] + nl * val[0]);
        const double Qsum = (sq_below[1] + nh * val[1] * val[1]) - (sq_below[0] + nl * val[0] * val[0]);
        const double mu = Ssum / (double)Ls;
        double var = (Qsum - Ssum * mu) / (double)(Ls - 1);
        if (var < 0) var = 0;
        params[2 * f] = (float)mu;
        params[2 * f + 1] = sqrtf((float)var + 1e-2f);
    }
}

// the selects as launches of their own (one workgroup per frame), for large batches: there the
// passes run many waves of workgroups, and a frame's select waiting for the frame's last slice
// delays the pass's tail (192 frames: 339 us with the selects folded in, 310 us as launches)
__global__ void __launch_bounds__(DS_SEL_T) k_ds_sel1(long long n, unsigned char* __restrict__ ws) {
    __shared__ __align__(16) unsigned h[DS_NB1];
    ds_sel1(blockIdx.x, n, ws, h);
}
__global__ void __launch_bounds__(DS_SEL_T) k_ds_sel2(long long n, int chunk, unsigned char* __restrict__ ws) {
    __shared__ __align__(16) unsigned h[2][DS_NB2];
    ds_sel2(blockIdx.x, n, chunk, ws, h);
}
__global__ void __launch_bounds__(DS_SEL_T) k_ds_fin(long long n, int chunk, unsigned char* __restrict__ ws,
                                                     float* __restrict__ params) {
    __shared__ __align__(16) unsigned h[2][DS_NB3];
    ds_fin(blockIdx.x, n, chunk, ws, params, h);
}

// ------------------------------------------------------------------------------------------
// normalise (+ optional back-projection of the same pixels, bf_backproject's arithmetic)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void ds_backproject1(const float* Ki, const float* RT, float x, int u, int v,
                                                float* xyz) {
    const float uvd[4] = {(float)u * x, (float)v * x, x, 1.0f};
    float cam[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        float a = Ki[4 * r] * uvd[0];
        a = a + Ki[4 * r + 1] * uvd[1];
        a = a + Ki[4 * r + 2] * uvd[2];
        a = a + Ki[4 * r + 3] * uvd[3];
        cam[r] = a;
    }
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        float a = RT[4 * r] * cam[0];
        a = a + RT[4 * r + 1] * cam[1];
        a = a + RT[4 * r + 2] * cam[2];
        a = a + RT[4 * r + 3] * cam[3];
        xyz[r] = a;
    }
}

template <int KV>
__global__ void __launch_bounds__(DS_T) k_ds_norm(const float* __restrict__ depth, int h, int w,
                                                  const float* __restrict__ params,
                                                  float* __restrict__ out, const float* __restrict__ K,
                                                  const float* __restrict__ RT, float max_depth,
                                                  float* __restrict__ xyz, uint8_t* __restrict__ valid) {
    constexpr int CHUNK = KV * 4 * DS_T;
    const long long n = (long long)h * w;
    const int s = blockIdx.x, f = blockIdx.y;
    const float* d = depth + (size_t)f * n;
    float4 v[KV];
    ds_load<KV>(d, n, s, v);
    float* o = out + (size_t)f * n;
    const float mean = params[2 * f], stdv = params[2 * f + 1];
    __shared__ float s_Ki[16], s_RT[16];
    __shared__ float4 s_xyz[(DS_T / 64) * 192];
    const bool bp = xyz != nullptr;
    if (bp) {
        if (threadIdx.x == 0) {
            const float* k = K + 9 * f;
            float K4[16] = {k[0], k[1], k[2], 0.f, k[3], k[4], k[5], 0.f, k[6], k[7], k[8], 0.f,
                            0.f, 0.f, 0.f, 1.f};
            bf_inv4(K4, s_Ki);
        }
        if (threadIdx.x < 16) s_RT[threadIdx.x] = RT[16 * f + threadIdx.x];
        __syncthreads();
    }
    float* xo = bp ? xyz + (size_t)f * n * 3 : nullptr;
    uint8_t* vo = bp ? valid + (size_t)f * n : nullptr;
    const long long base = (long long)s * CHUNK;
    // 4 consecutive pixels per thread and group: float4 out, and with the back-projection
    // 12 floats (3 x float4) + 4 valid bytes (one u32) per thread
    const bool vec = (n & 3) == 0 && w >= 4 && ((reinterpret_cast<uintptr_t>(d) & 15) == 0) &&
                     ((reinterpret_cast<uintptr_t>(o) & 15) == 0) &&
                     (!bp || (((reinterpret_cast<uintptr_t>(xo) & 15) == 0) &&
                              ((reinterpret_cast<uintptr_t>(vo) & 3) == 0)));
#pragma unroll
    for (int it = 0; it < KV; ++it) {
        const long long i0 = base + (long long)it * 4 * DS_T + 4 * threadIdx.x;
        const float x[4] = {v[it].x, v[it].y, v[it].z, v[it].w};
        if (vec) {
            // lanes past the frame (x = 0) run along so the wave's staged xyz copy stays whole
            const bool act = i0 < n;
            if (!__any(act)) continue;                         // wave-uniform
            float y[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) y[e] = ((ds_valid(x[e]) ? x[e] : mean) - mean) / stdv;
            if (act) *reinterpret_cast<float4*>(o + i0) = make_float4(y[0], y[1], y[2], y[3]);
            if (bp) {
                float p[12];
                unsigned vb = 0;
                const int u0 = (int)i0 % w, v0 = (int)i0 / w;       // (a frame is < 2^31 pixels)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    int u = u0 + e, vv = v0;
                    if (u >= w) { u -= w; vv += 1; }
                    ds_backproject1(s_Ki, s_RT, x[e], u, vv, p + 3 * e);
                    bool ok = x[e] > 0.f;
                    if (max_depth > 0.f) ok = ok && (x[e] < max_depth);
                    vb |= (ok ? 1u : 0u) << (8 * e);
                }
                // xyz through a per-wave LDS region: the wave's 64 x 48 B leave as 3 float4 per lane
                // along consecutive addresses (a lane's own 48 B at a 48-B stride would touch 3x
                // the lines per store instruction)
                float4* sw = s_xyz + (threadIdx.x >> 6) * 192;
                const int ln = threadIdx.x & 63;
                sw[3 * ln + 0] = make_float4(p[0], p[1], p[2], p[3]);
                sw[3 * ln + 1] = make_float4(p[4], p[5], p[6], p[7]);
                sw[3 * ln + 2] = make_float4(p[8], p[9], p[10], p[11]);
                // from the wave's first pixel: the float4s of the pixels inside the frame
                float4* xw = reinterpret_cast<float4*>(xo + 3 * (i0 - 4 * ln));
                const long long lim4 = 3 * (n - (i0 - 4 * ln)) / 4;
#pragma unroll
                for (int k2 = 0; k2 < 3; ++k2)
                    if (ln + 64 * k2 < lim4) xw[ln + 64 * k2] = sw[ln + 64 * k2];
                if (act) *reinterpret_cast<unsigned*>(vo + i0) = vb;
            }
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const long long i = i0 + e;
                if (i >= n) break;
                o[i] = ((ds_valid(x[e]) ? x[e] : mean) - mean) / stdv;
                if (bp) {
                    ds_backproject1(s_Ki, s_RT, x[e], (int)(i % w), (int)(i / w), xo + 3 * i);
                    bool ok = x[e] > 0.f;
                    if (max_depth > 0.f) ok = ok && (x[e] < max_depth);
                    vo[i] = ok ? 1 : 0;
                }
            }
        }
    }
}

BF_API size_t bf_depth_standardize_workspace_size(int b, int h, int w) {
    if (b <= 0 || h <= 0 || w <= 0) return 0;
    return (size_t)b * ds_layout((long long)h * w).stride;
}

template <int KV>
static void ds_launch(const float* depth, int b, int h, int w, float* out, float* params, const float* K,
                      const float* RT, float max_depth, float* xyz, uint8_t* valid, unsigned char* ws,
                      hipStream_t st) {
    constexpr int CHUNK = KV * 4 * DS_T;
    const long long n = (long long)h * w;
    const dim3 grid(ds_slices(n, CHUNK), b);
    if (KV == 4) {
        // small batches: three histogram passes, each with the frame's select run by its
        // last-arriving workgroup, then the normalise / back-projection pass -- four launches
        hipLaunchKernelGGL((k_ds_hist1<KV, true>), grid, dim3(DS_T), 0, st, depth, n, ws);
        hipLaunchKernelGGL((k_ds_hist2<KV, true>), grid, dim3(DS_T), 0, st, depth, n, ws);
        hipLaunchKernelGGL((k_ds_hist3<KV, true>), grid, dim3(DS_T), 0, st, depth, n, ws, params);
    } else {
        hipLaunchKernelGGL((k_ds_hist1<KV, false>), grid, dim3(DS_T), 0, st, depth, n, ws);
        hipLaunchKernelGGL(k_ds_sel1, dim3(b), dim3(DS_SEL_T), 0, st, n, ws);
        hipLaunchKernelGGL((k_ds_hist2<KV, false>), grid, dim3(DS_T), 0, st, depth, n, ws);
        hipLaunchKernelGGL(k_ds_sel2, dim3(b), dim3(DS_SEL_T), 0, st, n, CHUNK, ws);
        hipLaunchKernelGGL((k_ds_hist3<KV, false>), grid, dim3(DS_T), 0, st, depth, n, ws, params);
        hipLaunchKernelGGL(k_ds_fin, dim3(b), dim3(DS_SEL_T), 0, st, n, CHUNK, ws, params);
    }
    // the normalise pass carries no per-slice state: small batches run it on 2048-element slices
    // (four times the workgroups of the histogram passes), which it needs to keep enough stores in
    // flight across the chip
    constexpr int KVN = KV <= 4 ? DS_NORM_KV : KV;
    const dim3 ngrid(ds_slices(n, KVN * 4 * DS_T), b);
    hipLaunchKernelGGL(k_ds_norm<KVN>, ngrid, dim3(DS_T), 0, st, depth, h, w, params, out, K, RT, max_depth,
                       xyz, valid);
}

BF_API int bf_depth_preprocess(const float* depth, int b, int h, int w, float* out, float* params,
                               const float* K, const float* RT, float max_depth, float* xyz,
                               uint8_t* valid, void* workspace, void* stream) {
    if (b <= 0 || h <= 0 || w <= 0 || b > 65535 || !depth || !out || !params || !workspace)
        return BF_ERR_ARG;
    if (xyz && (!K || !RT || !valid)) return BF_ERR_ARG;
    const long long n = (long long)h * w;
    hipStream_t st = bf_stream(stream);
    unsigned char* ws = static_cast<unsigned char*>(workspace);
    // slices of 8192 elements while the batch gives fewer than ~1000 of them, else 32768
    // (16 float4 loads in flight per thread, a quarter of the workgroups)
    if ((long long)b * ds_slices(n, DS_MIN_CHUNK) >= 4096)
        ds_launch<16>(depth, b, h, w, out, params, K, RT, max_depth, xyz, valid, ws, st);
    else
        ds_launch<4>(depth, b, h, w, out, params, K, RT, max_depth, xyz, valid, ws, st);
    return bf_check_launch();
}

BF_API int bf_depth_standardize(const float* depth, int b, int h, int w, float* out, float* params,
                                void* workspace, void* stream) {
    return bf_depth_preprocess(depth, b, h, w, out, params, nullptr, nullptr, 0.0f, nullptr, nullptr,
                               workspace, stream);
}
