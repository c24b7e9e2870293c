// bf_jpeg.hip — baseline JPEG decode on the GPU (the colour half of frame
// ingestion): cv2.imread(color_path) of the reference's capture streams (capture_stream.py:194
// ScanNet, :402 CA-1M), i.e. libjpeg(-turbo)'s default decompression of a sequential Huffman JPEG:
// entropy decode (ITU T.81 F.2), dequantisation and the accurate integer IDCT (jidctint.c "islow"),
// fancy (triangle) upsampling of 4:2:0 / 4:2:2 chroma (jdsample.c, context rows replicated at the
// image edges) and the fixed-point YCbCr -> RGB tables of jdcolor.c.  Every step is integer
// arithmetic, so the result is checked for equality (oracle/jpeg.py, pinned to PIL's libjpeg-turbo).
//
// Four launches per batch of F files (device bytes back to back + F+1 offsets), all H x W:
//   k_jpeg_parse    one wave per file: markers (DQT, SOF0/1, DHT, DRI, SOS), the frame and scan
//                   layout, the entropy-coded segment's extent
//   k_jpeg_entropy  one wave per file (four per workgroup): the lanes un-stuff the entropy bytes (FF 00 -> FF, RSTn
//                   dropped) into an LDS ring 64 bytes per step; the Huffman walk runs wave-uniform
//                   (10-bit primary tables in LDS, a 16-bit canonical slow path), each block's
//                   coefficients gathered in LDS and stored by the 64 lanes (one int16 per lane)
//   k_jpeg_idct     one thread per 8 x 8 block: dequantise, islow IDCT, post-IDCT range limit
//   k_jpeg_color    four pixels per thread: fancy upsampling of the chroma planes + ycc -> RGB (u8 HWC)
#include "bf_common.h"

#define JPG_FB 10
#define JPG_RING 4096

struct JpegInfo {                 // per file, in the workspace (written by k_jpeg_parse)
    uint32_t nc, hmax, vmax, mcux, mcuy, dri, ent_off, ent_len;
    uint32_t h[3], v[3], tq[3], td[3], ta[3], bw[3], bh[3], coff[3];   // coff: block offset of the comp's grid
    uint16_t q[4][64];            // natural order
    uint8_t dht[8][16 + 256];     // DC 0-3, AC 4-7: counts[16], values
    uint32_t dht_mask, q_mask;
};

static inline size_t jpg_align(size_t v, size_t a) { return (v + a - 1) / a * a; }
__host__ __device__ inline uint32_t jpg_blocks_cap(int H, int W) {
    return 3u * (2u * (((uint32_t)H + 15) / 16)) * (2u * (((uint32_t)W + 15) / 16));
}

__device__ __forceinline__ uint32_t jrfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

__constant__ uint8_t jpg_zigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                       12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                       35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                       58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// ---- markers ----------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_jpeg_parse(const uint8_t* __restrict__ files, const int64_t* __restrict__ offs,
                                                   int F, int H, int W, JpegInfo* __restrict__ infos,
                                                   int32_t* __restrict__ status) {
    const int f = blockIdx.x;
    const int lane = threadIdx.x;
    if (f >= F) return;
    const uint8_t* p = files + offs[f];
    const long long n = offs[f + 1] - offs[f];
    JpegInfo* I = infos + f;
    int st = 0;
    bool frame = false, scan = false;
    uint32_t dht_mask = 0, q_mask = 0;
    if (n < 4 || p[0] != 0xFF || p[1] != 0xD8) st |= BF_JPG_BAD_MARKER;
    if (lane == 0) {
        I->dri = 0;
        I->nc = 0;
    }
    long long pos = 2;
    while (!st && !scan) {
        while (pos < n && p[pos] == 0xFF && pos + 1 < n && p[pos + 1] == 0xFF) ++pos;   // fill bytes
        if (pos + 4 > n || p[pos] != 0xFF) { st |= BF_JPG_BAD_MARKER; break; }
        const uint32_t m = p[pos + 1];
        if (m == 0xD9) { st |= BF_JPG_BAD_MARKER; break; }                              // EOI before SOS
        const uint32_t len = ((uint32_t)p[pos + 2] << 8) | p[pos + 3];
        if (len < 2 || pos + 2 + len > n) { st |= BF_JPG_BAD_MARKER; break; }
        const uint8_t* s = p + pos + 4;
        const uint32_t sl = len - 2;
        if (m == 0xDB) {                                                                 // DQT
            uint32_t i = 0;
            while (i < sl) {
                const uint32_t pq = s[i] >> 4, t = s[i] & 15;
                if (t > 3 || pq > 1 || i + 1 + (pq ? 128u : 64u) > sl) { st |= BF_JPG_BAD_MARKER; break; }
                const uint32_t zz = jpg_zigzag[lane];
                const uint32_t val = pq ? (((uint32_t)s[i + 1 + 2 * lane] << 8) | s[i + 2 + 2 * lane]) : s[i + 1 + lane];
                I->q[t][zz] = (uint16_t)val;
                q_mask |= 1u << t;
                i += 1 + (pq ? 128 : 64);
            }
        } else if (m == 0xC0 || m == 0xC1) {                                             // SOF0 / SOF1
            if (sl < 6) { st |= BF_JPG_BAD_MARKER; break; }
            const uint32_t prec = s[0], hh = ((uint32_t)s[1] << 8) | s[2], ww = ((uint32_t)s[3] << 8) | s[4], nc = s[5];
            if (prec != 8 || (nc != 1 && nc != 3) || sl < 6 + 3 * nc) { st |= BF_JPG_UNSUPPORTED; break; }
            if ((int)hh != H || (int)ww != W) st |= BF_JPG_SIZE;
            // a single-component scan is non-interleaved: one block per MCU whatever the factors say
            auto fh = [&](uint32_t c) -> uint32_t { return nc == 1 ? 1u : (uint32_t)(s[7 + 3 * c] >> 4); };
            auto fv = [&](uint32_t c) -> uint32_t { return nc == 1 ? 1u : (uint32_t)(s[7 + 3 * c] & 15); };
            uint32_t hm = 1, vm = 1;
            for (uint32_t c = 0; c < nc; ++c) {
                const uint32_t h = fh(c), v = fv(c), tq = s[8 + 3 * c];
                if (h < 1 || h > 2 || v < 1 || v > 2 || tq > 3) st |= BF_JPG_UNSUPPORTED;
                if (lane == 0) { I->h[c] = h; I->v[c] = v; I->tq[c] = tq; }
                hm = max(hm, h);
                vm = max(vm, v);
            }
            // luma at full resolution, chroma at full or half (h2v2 / h2v1 / h1v1 upsampling only)
            for (uint32_t c = 0; c < nc; ++c) {
                const uint32_t h = fh(c), v = fv(c);
                if (h == 0 || v == 0 || hm % h || vm % v || (vm / v == 2 && hm / h != 2)) st |= BF_JPG_UNSUPPORTED;
                if (c == 0 && (h != hm || v != vm)) st |= BF_JPG_UNSUPPORTED;
            }
            if (lane == 0) {
                I->nc = nc; I->hmax = hm; I->vmax = vm;
                I->mcux = (ww + 8 * hm - 1) / (8 * hm);
                I->mcuy = (hh + 8 * vm - 1) / (8 * vm);
                uint32_t off = 0;
                for (uint32_t c = 0; c < nc; ++c) {
                    const uint32_t h = fh(c), v = fv(c);
                    I->bw[c] = I->mcux * h;
                    I->bh[c] = I->mcuy * v;
                    I->coff[c] = off;
                    off += I->bw[c] * I->bh[c];
                }
            }
            frame = true;
        } else if (m >= 0xC2 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {       // progressive, lossless, arithmetic
            st |= BF_JPG_UNSUPPORTED;
        } else if (m == 0xC4) {                                                          // DHT
            uint32_t i = 0;
            while (i + 17 <= sl) {
                const uint32_t tc = s[i] >> 4, th = s[i] & 15;
                if (tc > 1 || th > 3) { st |= BF_JPG_BAD_MARKER; break; }
                uint32_t cnt = 0;
                for (int k = 0; k < 16; ++k) cnt += s[i + 1 + k];
                if (cnt > 256 || i + 17 + cnt > sl) { st |= BF_JPG_BAD_MARKER; break; }
                uint8_t* d = I->dht[tc * 4 + th];
                for (uint32_t k = lane; k < 16 + cnt; k += 64) d[k] = s[i + 1 + k];
                for (uint32_t k = 16 + cnt + lane; k < 16 + 256; k += 64) d[k] = 0;
                dht_mask |= 1u << (tc * 4 + th);
                i += 17 + cnt;
            }
        } else if (m == 0xDD) {                                                          // DRI
            if (sl < 2) { st |= BF_JPG_BAD_MARKER; break; }
            if (lane == 0) I->dri = ((uint32_t)s[0] << 8) | s[1];
        } else if (m == 0xDA) {                                                          // SOS
            if (!frame || sl < 1) { st |= BF_JPG_BAD_MARKER; break; }
            const uint32_t ns = s[0];
            uint32_t nc = 0;
            // one interleaved scan of every component (sequential JPEG as libjpeg / PIL write it)
            if (sl < 4 + 2 * ns) { st |= BF_JPG_BAD_MARKER; break; }
            nc = I->nc;
            if (ns != nc) { st |= BF_JPG_UNSUPPORTED; break; }
            for (uint32_t k = 0; k < ns; ++k) {
                const uint32_t td = s[2 + 2 * k] >> 4, ta = s[2 + 2 * k] & 15;
                if (td > 3 || ta > 3) st |= BF_JPG_BAD_MARKER;
                if (lane == 0) { I->td[k] = td; I->ta[k] = ta; }
            }
            const uint32_t ss = s[1 + 2 * ns], se = s[2 + 2 * ns], ahal = s[3 + 2 * ns];
            if (ss != 0 || se != 63 || ahal != 0) st |= BF_JPG_UNSUPPORTED;
            // entropy data: the rest of the file (the decode stops at the first marker that is
            // neither RSTn nor a stuffed FF)
            const long long e = pos + 2 + len;
            if (lane == 0) { I->ent_off = (uint32_t)e; I->ent_len = (uint32_t)(n - e); }
            scan = true;
        }
        pos += 2 + len;
    }
    if (!st && !scan) st |= BF_JPG_BAD_MARKER;
    if (lane == 0) {
        I->dht_mask = dht_mask;
        I->q_mask = q_mask;
        if (frame && scan) {
            if (!st) {
                for (uint32_t c = 0; c < I->nc; ++c)
                    if (!((q_mask >> I->tq[c]) & 1) || !((dht_mask >> I->td[c]) & 1) || !((dht_mask >> (4 + I->ta[c])) & 1))
                        st |= BF_JPG_BAD_MARKER;
            }
        }
        status[f] = st;
    }
}

// ---- entropy decode -----------------------------------------------------------------------------
// One wave per file.  The lanes un-stuff the entropy bytes into an LDS ring (JPG_SUB x 64 source
// bytes per refill, all loads in flight together; FF 00 -> FF, RSTn and fill bytes dropped, the
// first other marker ends the segment).  Decoding is speculative, as in the PNG inflate: each round, lane l
// decodes the token (Huffman code + its extra bits) that would start at bit P + l, once with each
// table a component of the scan uses (DC and AC); the scalar walk then follows the chain of real
// token starts through the per-lane results with v_readlane, across block and MCU boundaries, and
// ends the round at the first token starting past the 64 lanes.  A block's coefficients build up
// in one VGPR (lane i = natural index i) and are stored by the 64 lanes at its end.
#define JPG_SUB 8
#ifndef JPG_HALVES
#define JPG_HALVES 2                  // 64-bit halves of the stream decoded per round
#endif

#ifdef JPG_STATS
// diagnostic build (scripts/build_var.py jpg_stats -DJPG_STATS=1 bf_jpeg.hip): per file, the entropy
// kernel's shader-clock and 100-MHz stamps, rounds, tokens, slow tokens, refills, refill cycles, blocks
#define JPG_NSTAT 12
__device__ unsigned long long jpg_stats[4096 * JPG_NSTAT];
BF_API int bf_jpeg_read_stats(unsigned long long* dst, int n) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(jpg_stats), sizeof(unsigned long long) * JPG_NSTAT * n) == hipSuccess
               ? BF_OK : BF_ERR_LAUNCH;
}
#define JST(...) __VA_ARGS__
#else
#define JST(...)
#endif

struct JpegLds {
    uint16_t fast[8][1 << JPG_FB];    // (len << 8) | value for codes <= JPG_FB bits, 0 otherwise
    int32_t maxcode[8][18];           // jdhuff.c: largest code of each length (-1: none), [17] sentinel
    int32_t valoff[8][17];
    uint8_t vals[8][256];
    uint32_t ring[JPG_RING / 4];      // un-stuffed entropy bytes (byte writes, dword reads)
    int16_t blk[64];                  // the block being decoded, natural order
    uint8_t zz[80];                   // zigzag -> natural (64..79: 63, libjpeg's guard entries)
};

// canonical table (T.81 Annex C / jdhuff.c jpeg_make_d_derived_tbl) from counts + values
__device__ bool jpg_build(JpegLds& L, int t, const uint8_t* dht) {
    const int lane = threadIdx.x & 63;
    for (int i = lane; i < (1 << JPG_FB); i += 64) L.fast[t][i] = 0;
    for (int i = lane; i < 256; i += 64) L.vals[t][i] = dht[16 + i];
    __builtin_amdgcn_wave_barrier();  // (the tables are the wave's own: LDS order within a wave suffices)
    bool ok = true;
    {
        int code = 0;                 // over-subscribed tables (jdhuff.c "Bogus Huffman table") are refused
        for (int l = 1; l <= 16; ++l) {
            code += dht[l - 1];
            if (code > (1 << l)) ok = false;
            code <<= 1;
        }
    }
    if (lane == 0 && ok) {
        int code = 0, p = 0;
        for (int l = 1; l <= 16; ++l) {
            const int c = dht[l - 1];
            if (c) {
                L.valoff[t][l] = p - code;
                for (int k = 0; k < c; ++k, ++p, ++code) {
                    if (l <= JPG_FB) {
                        const int base = code << (JPG_FB - l);
                        for (int j = 0; j < (1 << (JPG_FB - l)); ++j)
                            L.fast[t][base + j] = (uint16_t)((l << 8) | dht[16 + p]);
                    }
                }
                L.maxcode[t][l] = code - 1;
            } else {
                L.maxcode[t][l] = -1;
                L.valoff[t][l] = 0;
            }
            code <<= 1;
        }
        L.maxcode[t][17] = 0x7fffffff;
    }
    __builtin_amdgcn_wave_barrier();
    return ok;
}

// 32 stream bits starting at bit q of the un-stuffed stream, MSB first
__device__ __forceinline__ uint32_t jpg_peek32(const JpegLds& L, uint32_t q) {
    const uint32_t d = (q >> 5) & (JPG_RING / 4 - 1);
    const uint32_t w0 = __builtin_bswap32(L.ring[d]);
    const uint32_t w1 = __builtin_bswap32(L.ring[(d + 1) & (JPG_RING / 4 - 1)]);
    return (uint32_t)((((uint64_t)w0 << 32) | w1) >> (32 - (q & 31)));
}

// the token at the head of `bits` with table t: packed (value int16 << 16) | flags | size << 9 |
// run << 5 | total bits (code + extra bits).  DC tokens: run 0, size = the magnitude category.
// jpg_token_fast answers from the 10-bit table only: a longer code gives JT_SLOW, decoded by the
// walk with jpg_token_slow if (rarely) the chain reaches that lane.
#define JT_BAD (1u << 13)
#define JT_SLOW (1u << 14)
__device__ __forceinline__ uint32_t jpg_pack(uint32_t bits, uint32_t len, uint32_t sym, bool dc) {
    const uint32_t run = dc ? 0u : (sym >> 4), sz = dc ? sym : (sym & 15u);
    if (sz > (dc ? 11u : 15u)) return JT_BAD;
    int val = 0;
    if (sz) {
        const uint32_t r = (bits << len) >> (32 - sz);
        val = r < (1u << (sz - 1)) ? (int)r - (1 << sz) + 1 : (int)r;
    }
    return ((uint32_t)val << 16) | (sz << 9) | (run << 5) | (len + sz);
}

__device__ __forceinline__ uint32_t jpg_token_fast(const JpegLds& L, int t, uint32_t bits, bool dc) {
    const uint32_t e = L.fast[t][bits >> (32 - JPG_FB)];
    return e ? jpg_pack(bits, e >> 8, e & 255u, dc) : JT_SLOW;
}

__device__ __noinline__ uint32_t jpg_token_slow(const JpegLds& L, int t, uint32_t bits, bool dc) {
    for (int l = JPG_FB + 1; l <= 16; ++l) {
        const int code = (int)(bits >> (32 - l));
        if (code <= L.maxcode[t][l]) return jpg_pack(bits, (uint32_t)l, L.vals[t][(code + L.valoff[t][l]) & 255], dc);
    }
    return JT_BAD;
}

// per-lane words of the walk from the 10-bit AC table entry ea of the token at bit P + lane:
//   aw  AC chain word: next token start (lane + bits, < 128) | (run + 1) << 8; EOB: 128 | next; slow: 255
//   av  AC coefficient: value << 16 | run << 1 | (size != 0)
__device__ __forceinline__ void jpg_lane_ac(uint32_t bits, uint32_t lane, uint32_t ea, uint32_t& aw, uint32_t& av) {
    const uint32_t len = ea >> 8, run = (ea >> 4) & 15u, sz = ea & 15u;
    uint32_t val = 0;
    if (sz) {
        const uint32_t r = (bits << len) >> (32 - sz);
        val = r < (1u << (sz - 1)) ? r - (1u << sz) + 1u : r;
    }
    const uint32_t nxt = lane + len + sz;
    aw = !ea ? 255u : (sz == 0 && run != 15) ? (128u | nxt) : (((run + 1) << 8) | nxt);
    av = (val << 16) | (run << 1) | (sz != 0);
}

// inclusive prefix sum over the wave (DPP row shifts + row broadcasts)
__device__ __forceinline__ uint32_t png_like_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);   // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

// JPG_WPB files per workgroup, one wave each with its own LDS: the waves land on the SIMDs of one
// CU, so a batch occupies F / JPG_WPB CUs instead of F (a full-CU GEMM workgroup cannot co-reside
// with a decode wave; in the pipeline every CU a decode holds is one the detector loses)
#define JPG_WPB 4
__global__ void __launch_bounds__(64 * JPG_WPB) k_jpeg_entropy(const uint8_t* __restrict__ files,
                                                               const int64_t* __restrict__ offs,
                                                               const JpegInfo* __restrict__ infos,
                                                               int16_t* __restrict__ coef, uint32_t blocks_cap,
                                                               int F, int32_t* __restrict__ status) {
    __shared__ JpegLds Ls[JPG_WPB];
    const uint32_t wv = jrfl(threadIdx.x >> 6);     // (wave-uniform; the compiler cannot tell by itself)
    JpegLds& L = Ls[wv];
    const int f = (int)(blockIdx.x * JPG_WPB + wv);
    const int lane = threadIdx.x & 63;
    if (f >= F || status[f]) return;
    const JpegInfo* I = infos + f;
    const uint8_t* ent = files + offs[f] + I->ent_off;
    const uint32_t elen = I->ent_len;
    const uint32_t nc = I->nc;
    int16_t* out = coef + (size_t)f * blocks_cap * 64;
    bool tables_ok = true;
    for (int t = 0; t < 8; ++t)
        if ((I->dht_mask >> t) & 1) tables_ok &= jpg_build(L, t, I->dht[t]);
    if (!tables_ok) {
        if (lane == 0) status[f] |= BF_JPG_BAD_MARKER;
        return;
    }
    uint8_t* ring8 = reinterpret_cast<uint8_t*>(L.ring);
    JST(const uint64_t c0 = __builtin_amdgcn_s_memtime(); const uint64_t r0 = __builtin_amdgcn_s_memrealtime();)
    JST(uint64_t n_rounds = 0, n_tok = 0, n_slow = 0, n_prod = 0, c_prod = 0, n_blk = 0, c_lanes = 0, c_walk = 0, n_seg = 0, c_post = 0;)

    // ---- producer: source position, bytes in the ring, last source byte, end of the data
    uint32_t sp = 0, prod = 0, prev = 0, real_end = 0xffffffffu;
    bool ended = false;
    auto produce = [&]() {
        if (ended) {                  // past the segment: zero bits (libjpeg's fill after a marker)
#pragma unroll
            for (int j = 0; j < JPG_SUB; ++j) ring8[(prod + j * 64 + lane) & (JPG_RING - 1)] = 0;
            prod += JPG_SUB * 64;
            return;
        }
        uint32_t b[JPG_SUB];
#pragma unroll
        for (int j = 0; j < JPG_SUB; ++j) {
            const uint32_t i = sp + j * 64 + lane;
            b[j] = i < elen ? ent[i] : 0u;
        }
        const uint32_t ti = sp + JPG_SUB * 64;
        const uint32_t tail = jrfl(ti < elen ? (uint32_t)ent[ti] : 0u);
#pragma unroll
        for (int j = 0; j < JPG_SUB; ++j) {
            const uint32_t i = sp + j * 64 + lane;
            // the shuffles run on all 64 lanes (a lane masked off during one reads back garbage)
            const uint32_t bu = (uint32_t)__shfl_up((int)b[j], 1, 64);
            const uint32_t bn = (uint32_t)__shfl_down((int)b[j], 1, 64);
            const uint32_t first = j == 0 ? prev : jrfl(__builtin_amdgcn_readlane(b[j - 1], 63));
            const uint32_t after = j + 1 < JPG_SUB ? jrfl(__builtin_amdgcn_readlane(b[j + 1], 0)) : tail;
            const uint32_t bp = lane == 0 ? first : bu;
            const uint32_t bx = lane == 63 ? after : bn;
            const bool valid = i < elen;
            const bool has_next = i + 1 < elen;
            const bool rst_next = bx >= 0xD0 && bx <= 0xD7;
            // a marker other than RSTn (FF xx, xx not 00) ends the entropy-coded segment
            // (FF FF: a fill byte -- jdhuff.c skips every FF of a run and reads what follows the last)
            const unsigned long long tm =
                __ballot(valid && has_next && b[j] == 0xFF && bx != 0 && bx != 0xFF && !rst_next);
            const uint32_t lim = tm ? (uint32_t)__builtin_ctzll(tm) : 64u;
            const bool stuffed = bp == 0xFF && b[j] == 0 && i > 0;
            const bool rst_ff = b[j] == 0xFF && has_next && rst_next;
            const bool rst_d = bp == 0xFF && b[j] >= 0xD0 && b[j] <= 0xD7 && i > 0;
            const bool fill = b[j] == 0xFF && has_next && bx == 0xFF;
            const bool keep = valid && (uint32_t)lane < lim && !stuffed && !rst_ff && !rst_d && !fill;
            const unsigned long long km = __ballot(keep);
            if (keep) ring8[(prod + (uint32_t)bf_lanes_below(km)) & (JPG_RING - 1)] = (uint8_t)b[j];
            prod += (uint32_t)__popcll(km);
            if (tm || sp + (uint32_t)(j + 1) * 64 >= elen) {   // (uniform: a lane-derived test here makes the whole walk divergent)
                ended = true;
                real_end = prod;      // un-stuffed bytes of real data
                break;
            }
        }
        prev = jrfl(__builtin_amdgcn_readlane(b[JPG_SUB - 1], 63));
        sp += JPG_SUB * 64;
        __builtin_amdgcn_wave_barrier();
    };

    // ---- scan layout
    uint32_t td[3], ta[3], hh[3], vv[3], bw[3], coff[3];
    for (uint32_t c = 0; c < 3; ++c) {
        const bool in = c < nc;
        td[c] = in ? I->td[c] : 0;
        ta[c] = in ? I->ta[c] : 0;
        hh[c] = in ? I->h[c] : 1;
        vv[c] = in ? I->v[c] : 1;
        bw[c] = in ? I->bw[c] : 0;
        coff[c] = in ? I->coff[c] : 0;
    }
    const uint32_t mcux = I->mcux, nmcu = mcux * I->mcuy, dri = I->dri;
    L.zz[lane] = (uint8_t)jpg_zigzag[lane];
    if (lane < 16) L.zz[64 + lane] = 63;
    L.blk[lane] = 0;

    // ---- walk state (uniform)
    uint32_t P = 0;                   // bit position of the next token in the un-stuffed stream
    uint32_t mcu = 0, mx = 0, my = 0, c = 0, bv = 0, bh = 0, k = 0;   // k == 0: the block's DC is next
    int pred0 = 0, pred1 = 0, pred2 = 0;
    bool insufficient = false, err = false;
    // the block's coefficients (LDS, natural order) -> its slot of the coefficient grid; re-zeroed
    auto store_block = [&]() {
        const size_t bi = (size_t)coff[c] + (size_t)(my * vv[c] + bv) * bw[c] + mx * hh[c] + bh;
        __builtin_amdgcn_wave_barrier();
        out[bi * 64 + lane] = L.blk[lane];
        L.blk[lane] = 0;
        __builtin_amdgcn_wave_barrier();
    };
    auto next_block = [&]() -> bool {  // true when a new MCU starts
        if (++bh < hh[c]) return false;
        bh = 0;
        if (++bv < vv[c]) return false;
        bv = 0;
        if (++c < nc) return false;
        c = 0;
        ++mcu;
        if (++mx == mcux) { mx = 0; ++my; }
        return true;
    };
    while (prod < 1024) produce();
    while (mcu < nmcu && !err) {
        if (insufficient) {           // zero MCU: zero blocks for each block of the MCU
            do {
                const size_t bi = (size_t)coff[c] + (size_t)(my * vv[c] + bv) * bw[c] + mx * hh[c] + bh;
                out[bi * 64 + lane] = 0;
            } while (!next_block());
        } else {
            JST(const uint64_t cp0 = __builtin_amdgcn_s_memtime();)
            while ((P >> 3) + 96 > prod) {
                produce();
                JST(++n_prod;)
            }
            JST(c_prod += __builtin_amdgcn_s_memtime() - cp0; ++n_rounds;)
            // ---- lanes: the AC tokens at P + lane (and P + 64 + lane: JPG_HALVES 64-bit halves per
            // round) with the table of the current block's component (DC tokens, one per block, are
            // decoded by the walk itself)
            const uint32_t rta = ta[c];
            const uint32_t bits0 = jpg_peek32(L, P + (uint32_t)lane);
#if JPG_HALVES > 1
            const uint32_t bits1 = jpg_peek32(L, P + 64u + (uint32_t)lane);
            const uint32_t fe1 = L.fast[4 + rta][bits1 >> (32 - JPG_FB)];
#endif
            const uint32_t fe0 = L.fast[4 + rta][bits0 >> (32 - JPG_FB)];
            uint32_t aw0, av0, aw1 = 0, av1 = 0;
            jpg_lane_ac(bits0, (uint32_t)lane, fe0, aw0, av0);
#if JPG_HALVES > 1
            jpg_lane_ac(bits1, (uint32_t)lane, fe1, aw1, av1);
#endif
            const uint32_t span = 64u * JPG_HALVES;
            JST(const uint64_t cw0 = __builtin_amdgcn_s_memtime(); c_lanes += cw0 - cp0;)
            // ---- the walk
            uint32_t at = 0;
            for (;;) {
                if (k == 0) {         // the block's DC token, wave-uniform
                    const uint32_t db = jrfl(jpg_peek32(L, P + at));
                    const uint32_t de = jrfl(L.fast[td[c]][db >> (32 - JPG_FB)]);
                    uint32_t inf = de ? jpg_pack(db, de >> 8, de & 255u, true) : jrfl(jpg_token_slow(L, (int)td[c], db, true));
                    JST(++n_tok;)
                    if (inf & JT_BAD) { err = true; break; }
                    at += inf & 31u;
                    int& pr = c == 0 ? pred0 : c == 1 ? pred1 : pred2;
                    pr += (int)inf >> 16;
                    if (lane == 0) L.blk[0] = (int16_t)pr;
                    k = 1;
                    if (at >= span) break;
                }
                if (ta[c] != rta) break;   // another AC table: the next round decodes with it
                bool done = false;
                for (;;) {            // AC segments: chain walks within a half, between slow tokens
                    const uint32_t hb = (JPG_HALVES > 1 && at >= 64) ? 64u : 0u;
                    const uint32_t aw = hb ? aw1 : aw0, av = hb ? av1 : av0;
                    uint64_t mem = 0;
                    const uint32_t k0 = k;
                    uint32_t a = at - hb, last, inf;
                    do {
                        mem |= 1ull << a;
                        last = a;
                        inf = jrfl(__builtin_amdgcn_readlane(aw, (int)a));
                        k = jrfl(k + (inf >> 8));     // (keeps the walk scalar: the compiler loses it otherwise)
                        a = inf & 255u;
                        JST(++n_tok;)
                    } while (a < 64 && k < 64);
                    const bool slow = (inf & 255u) == 255u, eob = !slow && (inf & 128u);
                    if (slow) mem &= ~(1ull << last);
                    JST(const uint64_t cq0 = __builtin_amdgcn_s_memtime(); ++n_seg;)
                    {                 // the chain's coefficients, in parallel: k of each = k0 + prefix
                        const bool in = (mem >> lane) & 1ull;
                        const uint32_t kin = in ? (aw >> 8) : 0u;
                        const uint32_t pos = k0 + png_like_scan(kin) - kin + ((av >> 1) & 15u);
                        const bool wr = in && (av & 1u);
                        // (the break stays out of the lane-divergent write: inside it, the compiler
                        // turns the whole walk into exec-masked vector code)
                        const bool bad = __ballot(wr && pos > 63) != 0;
                        if (wr && pos <= 63) L.blk[L.zz[pos]] = (int16_t)((int)av >> 16);
                        if (bad) err = true;
                    }
                    JST(__builtin_amdgcn_s_waitcnt(0); c_post += __builtin_amdgcn_s_memtime() - cq0;)
                    if (err) break;
                    if (eob) { at = hb + (inf & 127u); done = true; break; }
                    if (slow) {       // a code longer than JPG_FB bits: decoded here, wave-uniform
                        JST(++n_slow;)
                        const uint32_t t2 = jrfl(jpg_token_slow(L, 4 + (int)ta[c], jpg_peek32(L, P + hb + last), false));
                        if (t2 & JT_BAD) { err = true; break; }
                        at = hb + last + (t2 & 31u);
                        const uint32_t run = (t2 >> 5) & 15u, sz = (t2 >> 9) & 15u;
                        if (sz == 0 && run != 15) { done = true; break; }
                        k += run;
                        if (k > 63) {
                            if (sz) err = true;
                            done = true;
                            break;
                        }
                        if (sz && lane == 0) L.blk[L.zz[k]] = (int16_t)((int)t2 >> 16);
                        if (++k >= 64) { done = true; break; }
                        if (at >= span) break;
                        continue;
                    }
                    at = hb + a;
                    if (k >= 64) { done = true; break; }
                    if (at >= span) break;        // the round ends mid-block
                }                                 // (else the chain crossed into the next half)
                if (err || !done) break;
                JST(++n_blk;)
                store_block();
                k = 0;
                if (next_block()) {
                    if (mcu >= nmcu) break;
                    // a restart interval boundary, or decoding past the data: end the round here
                    const bool rst = dri && mcu % dri == 0;
                    const bool past = real_end != 0xffffffffu && P + at > real_end * 8u;
                    if (rst || past) {
                        P += at;
                        at = 0;
                        if (rst) {
                            P = (P + 7) & ~7u;   // byte-align; the RSTn bytes are not in the ring
                            pred0 = pred1 = pred2 = 0;
                            insufficient = false;
                        }
                        // jdhuff.c: once a decode has needed bits past the end of the data, the rest
                        // of the segment's MCUs are left zero (uniform grey), not decoded from the fill
                        if (real_end != 0xffffffffu && P > real_end * 8u) insufficient = true;
                        break;
                    }
                }
                if (at >= span) break;
            }
            JST(c_walk += __builtin_amdgcn_s_memtime() - cw0;)
            P += at;
            continue;
        }
        // after a zero MCU
        if (mcu < nmcu && dri && mcu % dri == 0) {
            P = (P + 7) & ~7u;
            pred0 = pred1 = pred2 = 0;
            insufficient = false;
        }
    }
    if (err && lane == 0) status[f] |= BF_JPG_BAD_DATA;
#ifdef JPG_STATS
    const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0 && f < 4096) {
        unsigned long long* o = jpg_stats + f * JPG_NSTAT;
        o[0] = c1 - c0; o[1] = r1 - r0; o[2] = n_rounds; o[3] = n_tok; o[4] = n_slow; o[5] = n_prod; o[6] = c_prod;
        o[7] = n_blk; o[8] = c_lanes; o[9] = c_walk; o[10] = n_seg; o[11] = c_post;
    }
#endif
}

// ---- IDCT (jidctint.c jpeg_idct_islow) ----------------------------------------------------------
#define JI_CB 13
#define JI_P1 2
#define JFIX(x) ((int)((x) * (1 << JI_CB) + 0.5))

// the post-IDCT range-limit table of jdmaster.c, indexed by v & 1023 (v centred at 0)
__device__ __forceinline__ uint32_t jpg_range(int v) {
    const int i = v & 1023;
    return i < 128 ? (uint32_t)(i + 128) : (i < 512 ? 255u : (i < 896 ? 0u : (uint32_t)(i - 896)));
}

__device__ __forceinline__ void jpg_idct_1d(const long long z[8], long long o[8]) {
    // even part
    const long long z1e = (z[2] + z[6]) * JFIX(0.541196100);
    const long long t2 = z1e + z[6] * (-JFIX(1.847759065));
    const long long t3 = z1e + z[2] * JFIX(0.765366865);
    const long long t0 = (z[0] + z[4]) * (1 << JI_CB);
    const long long t1 = (z[0] - z[4]) * (1 << JI_CB);
    const long long t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
    // odd part
    long long o0 = z[7], o1 = z[5], o2 = z[3], o3 = z[1];
    long long zz1 = o0 + o3, zz2 = o1 + o2, zz3 = o0 + o2, zz4 = o1 + o3;
    const long long zz5 = (zz3 + zz4) * JFIX(1.175875602);
    o0 *= JFIX(0.298631336);
    o1 *= JFIX(2.053119869);
    o2 *= JFIX(3.072711026);
    o3 *= JFIX(1.501321110);
    zz1 *= -JFIX(0.899976223);
    zz2 *= -JFIX(2.562915447);
    zz3 = zz3 * (-JFIX(1.961570560)) + zz5;
    zz4 = zz4 * (-JFIX(0.390180644)) + zz5;
    o0 += zz1 + zz3;
    o1 += zz2 + zz4;
    o2 += zz2 + zz3;
    o3 += zz1 + zz4;
    o[0] = t10 + o3; o[7] = t10 - o3;
    o[1] = t11 + o2; o[6] = t11 - o2;
    o[2] = t12 + o1; o[5] = t12 - o1;
    o[3] = t13 + o0; o[4] = t13 - o0;
}

__global__ void __launch_bounds__(256) k_jpeg_idct(const JpegInfo* __restrict__ infos, const int16_t* __restrict__ coef,
                                                   uint32_t blocks_cap, int F, uint8_t* __restrict__ planes,
                                                   const int32_t* __restrict__ status) {
    const int f = blockIdx.y;
    if (f >= F || status[f]) return;
    const JpegInfo* I = infos + f;
    const uint32_t nc = I->nc;
    uint32_t total = 0;
    for (uint32_t c = 0; c < nc; ++c) total += I->bw[c] * I->bh[c];
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= total) return;
    uint32_t c = 0;
    while (c + 1 < nc && b >= I->coff[c + 1]) ++c;
    const uint32_t local = b - I->coff[c], by = local / I->bw[c], bx = local - by * I->bw[c];
    const int16_t* src = coef + ((size_t)f * blocks_cap + b) * 64;
    const uint16_t* q = I->q[I->tq[c]];
    int ws[64];
#pragma unroll
    for (int u = 0; u < 8; ++u) {                      // pass 1: columns
        long long z[8], o[8];
#pragma unroll
        for (int v = 0; v < 8; ++v) z[v] = (int)src[v * 8 + u] * (int)q[v * 8 + u];
        jpg_idct_1d(z, o);
#pragma unroll
        for (int v = 0; v < 8; ++v) ws[v * 8 + u] = (int)((o[v] + (1 << (JI_CB - JI_P1 - 1))) >> (JI_CB - JI_P1));
    }
    uint8_t* plane = planes + ((size_t)f * blocks_cap + I->coff[c]) * 64;   // the comp's plane: bh*8 x bw*8
    const uint32_t pw = I->bw[c] * 8;
#pragma unroll
    for (int v = 0; v < 8; ++v) {                      // pass 2: rows
        long long z[8], o[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) z[u] = ws[v * 8 + u];
        jpg_idct_1d(z, o);
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint32_t s = jpg_range((int)((o[u] + (1 << (JI_CB + JI_P1 + 3 - 1))) >> (JI_CB + JI_P1 + 3)));
            if (u < 4) lo |= s << (8 * u); else hi |= s << (8 * (u - 4));
        }
        uint2* dst = reinterpret_cast<uint2*>(plane + (size_t)(by * 8 + v) * pw + bx * 8);
        *dst = make_uint2(lo, hi);
    }
}

// ---- upsampling + colour conversion ----------------------------------------------------------
// chroma sample of the fancy upsampler (jdsample.c h2v2 / h2v1; fullsize copy) at output (x, y)
__device__ __forceinline__ int jpg_chroma(const uint8_t* pl, uint32_t pw, int cw, int ch, int rx, int ry, int x, int y) {
    if (rx == 1 && ry == 1) return pl[(size_t)y * pw + x];
    // the triangle filter with the neighbour column (and row) clamped at the plane's edges: at an
    // edge that reproduces jdsample.c's special cases exactly ((4p + 1) >> 2 = p for h2v1, the
    // (4s + 8) >> 4 / (4s + 7) >> 4 end columns for h2v2), so no branch is needed
    const int c = x >> 1, e = x & 1;
    const int cn = e ? min(c + 1, cw - 1) : max(c - 1, 0);
    auto S = [&](int col, int row) -> int { return pl[(size_t)row * pw + col]; };
    if (ry == 1) return (3 * S(c, y) + S(cn, y) + 1 + e) >> 2;               // h2v1_fancy_upsample
    const int r = y >> 1;                                                     // h2v2_fancy_upsample:
    const int rn = (y & 1) ? min(r + 1, ch - 1) : max(r - 1, 0);             // column sums with the row
    const int sc = 3 * S(c, r) + S(c, rn), sn = 3 * S(cn, r) + S(cn, rn);   // above / below
    return (3 * sc + sn + 8 - e) >> 4;
}

// jdcolor.c ycc_rgb_convert (SCALEBITS 16) of one pixel -> packed 0x00BBGGRR
__device__ __forceinline__ uint32_t jpg_ycc_rgb(int Y, int cbs, int crs) {
    const int cb = cbs - 128, cr = crs - 128;
    const int half = 1 << 15;
    const int r = Y + ((91881 * cr + half) >> 16);                    // FIX(1.40200) = 91881
    const int g = Y + (((-22554) * cb + half + (-46802) * cr) >> 16); // FIX(0.34414) = 22554, FIX(0.71414) = 46802
    const int b = Y + ((116130 * cb + half) >> 16);                   // FIX(1.77200) = 116130
    return (uint32_t)min(max(r, 0), 255) | ((uint32_t)min(max(g, 0), 255) << 8) | ((uint32_t)min(max(b, 0), 255) << 16);
}

// four consecutive pixels (row-major over the image) per thread, written as three dwords
__global__ void __launch_bounds__(256) k_jpeg_color(const JpegInfo* __restrict__ infos, const uint8_t* __restrict__ planes,
                                                    uint32_t blocks_cap, int F, int H, int W, uint8_t* __restrict__ rgb,
                                                    const int32_t* __restrict__ status) {
    const int f = blockIdx.y;
    if (f >= F || status[f]) return;
    const uint32_t HW = (uint32_t)H * (uint32_t)W;
    const uint32_t p0 = 4u * (blockIdx.x * blockDim.x + threadIdx.x);
    if (p0 >= HW) return;
    const JpegInfo* I = infos + f;
    const uint8_t* base = planes + (size_t)f * blocks_cap * 64;
    const uint8_t* yp = base + (size_t)I->coff[0] * 64;
    const uint32_t yw = I->bw[0] * 8;
    const bool grey = I->nc == 1;
    const uint8_t* cp[2] = {base, base};
    uint32_t pw[2] = {0, 0};
    int rx[2] = {1, 1}, ry[2] = {1, 1}, cw[2] = {1, 1}, chh[2] = {1, 1};
    if (!grey) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint32_t c = 1 + k;
            rx[k] = (int)(I->hmax / I->h[c]);
            ry[k] = (int)(I->vmax / I->v[c]);
            cw[k] = (int)((W * I->h[c] + I->hmax - 1) / I->hmax);
            chh[k] = (int)((H * I->v[c] + I->vmax - 1) / I->vmax);
            cp[k] = base + (size_t)I->coff[c] * 64;
            pw[k] = I->bw[c] * 8;
        }
    }
    int y = (int)(p0 / (uint32_t)W), x = (int)(p0 - (uint32_t)y * W);
    uint32_t px[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        uint32_t v = 0;
        if (p0 + j < HW) {
            const int Y = yp[(size_t)y * yw + x];
            if (grey) {
                v = (uint32_t)Y * 0x010101u;
            } else {
                const int cb = jpg_chroma(cp[0], pw[0], cw[0], chh[0], rx[0], ry[0], x, y);
                const int cr = jpg_chroma(cp[1], pw[1], cw[1], chh[1], rx[1], ry[1], x, y);
                v = jpg_ycc_rgb(Y, cb, cr);
            }
        }
        px[j] = v;
        if (++x == W) { x = 0; ++y; }
    }
    const size_t o = ((size_t)f * HW + p0) * 3;
    if (p0 + 3 < HW && (o & 3) == 0) {
        uint32_t* d = reinterpret_cast<uint32_t*>(rgb + o);
        d[0] = px[0] | (px[1] << 24);
        d[1] = (px[1] >> 8) | (px[2] << 16);
        d[2] = (px[2] >> 16) | (px[3] << 8);
    } else {
        for (int j = 0; j < 4 && p0 + j < HW; ++j) {
            rgb[o + 3 * j] = (uint8_t)px[j];
            rgb[o + 3 * j + 1] = (uint8_t)(px[j] >> 8);
            rgb[o + 3 * j + 2] = (uint8_t)(px[j] >> 16);
        }
    }
}

BF_API size_t bf_jpeg_workspace_bytes(int F, int H, int W) {
    if (F < 0 || H <= 0 || W <= 0) return 0;
    const size_t cap = jpg_blocks_cap(H, W);
    return jpg_align((size_t)F * sizeof(JpegInfo), 256) + jpg_align((size_t)F * cap * 64 * 2, 256) +
           jpg_align((size_t)F * cap * 64, 256);
}

BF_API int bf_jpeg_decode_rgb(const uint8_t* files, const int64_t* offsets, int F, int H, int W, uint8_t* rgb,
                              void* work, size_t work_bytes, int32_t* status, void* stream) {
    if (!files || !offsets || !rgb || !work || !status || F < 0 || H <= 0 || W <= 0) return BF_ERR_ARG;
    if (H > 16384 || W > 16384) return BF_ERR_UNSUPPORTED;
    if (work_bytes < bf_jpeg_workspace_bytes(F, H, W)) return BF_ERR_CAPACITY;
    if (F == 0) return BF_OK;
    const uint32_t cap = jpg_blocks_cap(H, W);
    uint8_t* w = static_cast<uint8_t*>(work);
    JpegInfo* infos = reinterpret_cast<JpegInfo*>(w);
    int16_t* coef = reinterpret_cast<int16_t*>(w + jpg_align((size_t)F * sizeof(JpegInfo), 256));
    uint8_t* planes = w + jpg_align((size_t)F * sizeof(JpegInfo), 256) + jpg_align((size_t)F * cap * 64 * 2, 256);
    hipStream_t s = bf_stream(stream);
    hipLaunchKernelGGL(k_jpeg_parse, dim3(F), dim3(64), 0, s, files, offsets, F, H, W, infos, status);
    hipLaunchKernelGGL(k_jpeg_entropy, dim3((F + JPG_WPB - 1) / JPG_WPB), dim3(64 * JPG_WPB), 0, s, files, offsets,
                       infos, coef, cap, F, status);
    hipLaunchKernelGGL(k_jpeg_idct, dim3((cap + 255) / 256, F), dim3(256), 0, s, infos, coef, cap, F, planes, status);
    const unsigned gp = (unsigned)(((size_t)H * W + 1023) / 1024);
    hipLaunchKernelGGL(k_jpeg_color, dim3(gp, F), dim3(256), 0, s, infos, planes, cap, F, H, W, rgb, status);
    return bf_check_launch();
}
