// bf_png.hip — 16-bit depth PNG decode on the GPU (the decode half of frame
// ingestion): cv2.imread(depth_path, cv2.IMREAD_UNCHANGED) of the reference's capture streams
// (capture_stream.py:197 ScanNet, :405 CA-1M) for the files those datasets ship — greyscale,
// 16 bits per sample, not interlaced.  PNG is lossless, so the result is defined bit for bit by
// the file (RFC 1950 zlib / RFC 1951 deflate / PNG 1.2 filtering); any other image kind is
// reported, not decoded.
//
// Four launches per batch of F files (device bytes of the files back to back + F+1 offsets):
//   k_png_parse    one wave per file walks the chunk list: signature, IHDR, the IDAT segments
//   k_png_gather   copies each file's IDAT payloads into one contiguous, 16-B aligned zlib stream
//   k_png_inflate  one wave per file decodes the stream: the Huffman / LZ77 walk is serial by
//                  construction and runs wave-uniform (scalar bit reader, table entries in LDS
//                  read by broadcast), the match copies run on the 64 lanes, the output goes
//                  through a 64 KiB LDS window that the lanes flush to HBM in 16 KiB pieces, and
//                  the Adler-32 of the inflated bytes is summed during those flushes
//   k_png_unfilter one wave per file undoes the per-row filters (None / Sub / Up / Average /
//                  Paeth on 2-byte pixels) on a diagonal wavefront: lane l holds row b0 + l and
//                  runs one pixel behind lane l - 1, so the row above arrives by a lane shift
// Status per file (int32, BF_PNG_* bits) says what was wrong with a file that did not decode.
#include "bf_common.h"

#define PNG_FB 11                 // primary Huffman table bits (longer codes: the bit-serial path)
#define PNG_RING (1 << 16)        // LDS output window (deflate needs the last 32 KiB)
#define PNG_FLUSH (1 << 14)
#ifndef PNG_HALVES
#define PNG_HALVES 2              // candidate token starts per round: 64 per half (one per lane)
#endif

struct PngSegTable {              // per file, in the workspace
    uint32_t nseg, zlen, width, height;
};
struct PngSeg {                   // one IDAT chunk: logical start in the zlib stream, byte offset in the file
    uint32_t zstart, phys;
};
// file f's IDAT list starts at entry offsets[f] / 12 + f of the segment array: a chunk takes at
// least 12 file bytes, so no file's list reaches the next file's (any number of IDAT chunks)
__host__ __device__ inline long long png_seg0(long long file_off, int f) { return file_off / 12 + f; }

static inline size_t png_align(size_t v, size_t a) { return (v + a - 1) / a * a; }

// workspace: [F seg tables][IDAT lists][zlib streams: file f at zoff(f)][filtered rows F x H x (2W+1)]
static inline size_t png_tab_bytes(int F) { return png_align((size_t)F * sizeof(PngSegTable), 256); }
static inline size_t png_list_bytes(int F, long long total) {
    return png_align(((size_t)total / 12 + (size_t)F + 1) * sizeof(PngSeg), 256);
}
static inline size_t png_z_bytes(int F, long long total) { return png_align((size_t)total + 32 * (size_t)F + 64, 256); }
// filtered rows of one file: H x (2W + 1) bytes, each file's block 16-B aligned
__host__ __device__ inline uint64_t png_rstride(int H, int W) { return ((uint64_t)H * (2 * (uint64_t)W + 1) + 15) & ~15ull; }
__host__ __device__ inline long long png_zoff(long long file_off, int f) { return ((file_off + 15) & ~15ll) + 32ll * f; }

__device__ __forceinline__ uint32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

#ifdef PNG_STATS
// diagnostic build (scripts/build_var.py png_stats -DPNG_STATS=1 bf_png.hip): per file, the inflate's
// shader-clock and 100-MHz stamps, rounds, tokens, bit-serial tokens, matches; the unfilter's stamps
#define PNG_NSTAT 10
__device__ unsigned long long png_stats[4096 * PNG_NSTAT];
BF_API int bf_png_read_stats(unsigned long long* dst, int n) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(png_stats), sizeof(unsigned long long) * PNG_NSTAT * n) == hipSuccess
               ? BF_OK : BF_ERR_LAUNCH;
}
#endif

__device__ __forceinline__ uint32_t ld_be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

// ---- chunk walk ----------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_png_parse(const uint8_t* __restrict__ files, const int64_t* __restrict__ offs,
                                                  int F, int H, int W, PngSegTable* __restrict__ tabs,
                                                  PngSeg* __restrict__ segs, int32_t* __restrict__ status) {
    const int f = blockIdx.x;
    if (f >= F) return;
    const long long base = offs[f], end = offs[f + 1];
    const uint8_t* p = files + base;
    const long long n = end - base;
    PngSegTable* T = tabs + f;
    PngSeg* S = segs + png_seg0(base, f);
    int st = 0;
    uint32_t nseg = 0, zlen = 0;
    const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (n < 8 + 25 + 12) st |= BF_PNG_BAD_SIGNATURE;
    for (int i = 0; i < 8 && !st; ++i)
        if (p[i] != sig[i]) st |= BF_PNG_BAD_SIGNATURE;
    if (!st) {
        long long pos = 8;
        bool seen_ihdr = false, seen_iend = false;
        while (pos + 12 <= n && !seen_iend && !st) {
            const uint32_t len = ld_be32(p + pos);
            const uint32_t type = ld_be32(p + pos + 4);
            if (len > 0x7fffffffu || pos + 12 + (long long)len > n) { st |= BF_PNG_BAD_CHUNK; break; }
            const uint8_t* d = p + pos + 8;
            if (!seen_ihdr) {
                if (type != 0x49484452u || len != 13) { st |= BF_PNG_BAD_HEADER; break; }   // IHDR first
                const uint32_t w = ld_be32(d), h = ld_be32(d + 4);
                if (w == 0 || h == 0 || d[10] != 0 || d[11] != 0) { st |= BF_PNG_BAD_HEADER; break; }
                if (d[8] != 16 || d[9] != 0 || d[12] != 0) st |= BF_PNG_UNSUPPORTED;      // 16-bit grey only
                if ((int)w != W || (int)h != H) st |= BF_PNG_SIZE;
                seen_ihdr = true;
            } else if (type == 0x49444154u) {            // IDAT
                if (len) {
                    if ((uint64_t)zlen + len >= (1ull << 31)) { st |= BF_PNG_BAD_CHUNK; break; }
                    if (threadIdx.x == 0) S[nseg] = PngSeg{zlen, (uint32_t)(pos + 8)};
                    ++nseg;
                    zlen += len;
                }
            } else if (type == 0x49454e44u) {            // IEND
                seen_iend = true;
            } else if (!(type & 0x20000000u)) {           // unknown critical chunk (PLTE is meaningless here)
                if (type != 0x504c5445u) st |= BF_PNG_UNSUPPORTED;
            }
            pos += 12 + (long long)len;
        }
        if (!seen_ihdr && !st) st |= BF_PNG_BAD_HEADER;
        if (nseg == 0 && !st) st |= BF_PNG_BAD_CHUNK;
    }
    if (threadIdx.x == 0) {
        T->nseg = st ? 0 : nseg;
        T->zlen = st ? 0 : zlen;
        T->width = W;
        T->height = H;
        status[f] = st;
    }
}

// ---- IDAT payloads -> one contiguous stream per file (16 bytes per thread) -----------------
__global__ void __launch_bounds__(256) k_png_gather(const uint8_t* __restrict__ files, const int64_t* __restrict__ offs,
                                                    const PngSegTable* __restrict__ tabs, const PngSeg* __restrict__ segs,
                                                    uint8_t* __restrict__ z) {
    const int f = blockIdx.y;
    const PngSegTable* T = tabs + f;
    const PngSeg* S = segs + png_seg0(offs[f], f);
    const uint32_t zlen = T->zlen, nseg = T->nseg;
    const uint32_t q0 = ((uint32_t)blockIdx.x * 256 + threadIdx.x) * 16;
    if (q0 >= zlen + 16) return;
    const uint8_t* src = files + offs[f];
    uint8_t* dst = z + png_zoff(offs[f], f) + q0;
    // segment holding q0: last s with zstart[s] <= q0
    uint32_t lo = 0, hi = nseg;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (S[mid].zstart <= q0) lo = mid; else hi = mid;
    }
    uint32_t s = lo;
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t q = q0 + j;
        uint32_t b = 0;
        if (q < zlen) {
            while (s + 1 < nseg && S[s + 1].zstart <= q) ++s;
            b = src[S[s].phys + (q - S[s].zstart)];
        }
        w[j >> 2] |= b << (8 * (j & 3));
    }
    *reinterpret_cast<uint4*>(dst) = make_uint4(w[0], w[1], w[2], w[3]);
}

// ---- inflate --------------------------------------------------------------------------------
struct PngBits {                  // LSB-first bit reader over 32-bit words, wave-uniform state
    const uint32_t* z;
    uint32_t idx, lim, nb;
    uint64_t buf;
    __device__ __forceinline__ void need() {
        if (nb < 32) {
            const uint32_t i = idx < lim ? idx : lim;
            buf |= (uint64_t)z[i] << nb;
            ++idx;
            nb += 32;
        }
    }
    __device__ __forceinline__ uint32_t peek(int n) const { return (uint32_t)buf & ((1u << n) - 1u); }
    __device__ __forceinline__ void drop(int n) { buf >>= n; nb -= n; }
    __device__ __forceinline__ uint32_t get(int n) { need(); const uint32_t v = peek(n); drop(n); return v; }
    __device__ __forceinline__ uint64_t consumed() const { return (uint64_t)idx * 32 - nb; }
    __device__ __forceinline__ void seek_bit(uint32_t bit) {
        idx = bit >> 5;
        const uint32_t i = idx < lim ? idx : lim;
        const int sh = (int)(bit & 31);
        buf = (uint64_t)(z[i] >> sh);
        nb = 32 - sh;
        ++idx;
    }
    __device__ __forceinline__ void seek_byte(uint64_t byte) {
        idx = (uint32_t)(byte >> 2);
        const uint32_t i = idx < lim ? idx : lim;
        const int sh = 8 * (int)(byte & 3);
        buf = (uint64_t)(z[i] >> sh);
        nb = 32 - sh;
        ++idx;
    }
};

struct PngLds {
    __attribute__((aligned(16))) uint8_t ring[PNG_RING];
    uint16_t lit[1 << PNG_FB];
    uint16_t dist[1 << PNG_FB];
    uint16_t lsym[288], dsym[32];
    uint16_t lcnt[16], dcnt[16];
    uint16_t ncode[16], noff[16];
    uint8_t lens[320];
};

// canonical Huffman code of lens[0..n) (RFC 1951 §3.2.2) -> primary table (sym << 4 | len for
// codes of <= PNG_FB bits, 0 otherwise), counts and the symbols sorted by (length, symbol) for the
// bit-serial slow path.  kind 0 = code-length code (must be complete), 1 = lit/len or distance
// (incomplete only as a single 1-bit code, zlib's inflate_table rule).  Returns false on an
// over-subscribed / invalid set.
__device__ bool png_build(PngLds& L, const uint8_t* lens, int n, uint16_t* table, uint16_t* cnt, uint16_t* sorted,
                          int kind) {
    const int lane = threadIdx.x;
    uint32_t run[16];
#pragma unroll
    for (int v = 0; v < 16; ++v) run[v] = 0;
    for (int c = 0; c < n; c += 64) {
        const int s = c + lane;
        const int len = s < n ? lens[s] : 0;
#pragma unroll
        for (int v = 1; v < 16; ++v) run[v] += __popcll(__ballot(len == v));
    }
    int left = 1, maxlen = 0;
#pragma unroll
    for (int v = 1; v < 16; ++v) {
        left = (left << 1) - (int)run[v];
        if (run[v]) maxlen = v;
    }
    if (left < 0) return false;
    if (left > 0 && maxlen != 0 && (kind == 0 || maxlen != 1)) return false;
    if (lane == 0) {
        uint32_t code = 0, off = 0;
        cnt[0] = 0;
#pragma unroll
        for (int v = 1; v < 16; ++v) {
            code = (code + (v > 1 ? run[v - 1] : 0)) << 1;
            L.ncode[v] = (uint16_t)code;
            L.noff[v] = (uint16_t)off;
            cnt[v] = (uint16_t)run[v];
            off += run[v];
        }
    }
    for (int i = lane; i < (1 << PNG_FB); i += 64) table[i] = 0;
    __syncthreads();
#pragma unroll
    for (int v = 0; v < 16; ++v) run[v] = 0;
    for (int c = 0; c < n; c += 64) {
        const int s = c + lane;
        const int len = s < n ? lens[s] : 0;
        uint32_t rank = 0;
#pragma unroll
        for (int v = 1; v < 16; ++v) {
            const unsigned long long m = __ballot(len == v);
            if (len == v) rank = run[v] + bf_lanes_below(m);
            run[v] += __popcll(m);
        }
        if (len) {
            const uint32_t code = L.ncode[len] + rank;
            sorted[L.noff[len] + rank] = (uint16_t)s;
            if (len <= PNG_FB) {
                const uint32_t r = __builtin_bitreverse32(code) >> (32 - len);
                const uint16_t e = (uint16_t)((s << 4) | len);
                for (uint32_t j = 0; j < (1u << (PNG_FB - len)); ++j) table[r | (j << len)] = e;
            }
        }
    }
    __syncthreads();
    return true;
}

// one symbol: table hit, or the bit-serial canonical walk (puff.c's decode) for long codes.
// Returns -1 for a bit pattern that is no code of the set.
__device__ __forceinline__ int png_decode(PngBits& br, const uint16_t* table, const uint16_t* cnt,
                                          const uint16_t* sorted) {
    br.need();
    const uint32_t e = rfl(table[br.peek(PNG_FB)]);
    if (e & 15) {
        br.drop(e & 15);
        return (int)(e >> 4);
    }
    int code = 0, first = 0, index = 0;
#pragma unroll 1
    for (int len = 1; len < 16; ++len) {
        code |= (int)br.get(1);
        const int count = (int)rfl(cnt[len]);
        if (code < first + count) return (int)rfl(sorted[index + (code - first)]);
        index += count;
        first = (first + count) << 1;
        code <<= 1;
    }
    return -1;
}

// inclusive prefix sum over the 64 lanes (DPP: row shifts, then the row broadcasts of GFX9)
__device__ __forceinline__ uint32_t png_wave_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);   // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

// flush ring bytes [from, to) (from 16-B aligned) to out; Adler-32 sums of the bytes < total
__device__ __forceinline__ void png_flush(PngLds& L, uint8_t* __restrict__ out, uint32_t from, uint32_t to,
                                          uint32_t total, uint64_t& s1, uint64_t& s2) {
    __syncthreads();
    for (uint32_t p = from + 16 * (uint32_t)threadIdx.x; p < to; p += 16 * 64) {
        const uint4 v = *reinterpret_cast<const uint4*>(&L.ring[p & (PNG_RING - 1)]);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t q = p + j;
            const uint32_t b = (w[j >> 2] >> (8 * (j & 3))) & 255u;
            if (q < to && q < total) {
                s1 += b;
                s2 += (uint64_t)q * b;
            }
        }
        if (p + 16 <= total) {
            *reinterpret_cast<uint4*>(out + p) = v;
        } else {
            for (int j = 0; j < 16; ++j)
                if (p + j < total) out[p + j] = (uint8_t)((w[j >> 2] >> (8 * (j & 3))) & 255u);
        }
    }
}

// `n` (<= 32) bits of the stream at bit P (LSB first), wave-uniform
__device__ __forceinline__ uint32_t png_bits(const uint32_t* z, uint32_t lim, uint32_t P, int n) {
    const uint32_t i = P >> 5;
    const uint64_t w = (uint64_t)z[min(i, lim)] | ((uint64_t)z[min(i + 1, lim)] << 32);
    return (uint32_t)(w >> (P & 31)) & (n >= 32 ? 0xffffffffu : ((1u << n) - 1u));
}

// The rarely taken parts of the inflate walk live in functions of their own (not inlined), so the
// register allocation of the round loop below is not shaped by them (inlined, they pushed the
// kernel to the 106-SGPR limit and spilled ~600 SGPR values into VGPR lanes in the loop).

// fixed Huffman codes (RFC 1951 §3.2.6)
__device__ __noinline__ void png_tables_fixed(PngLds* L) {
    for (int i = threadIdx.x; i < 320; i += 64)
        L->lens[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : i < 288 ? 8 : 5;
    __syncthreads();
    png_build(*L, L->lens, 288, L->lit, L->lcnt, L->lsym, 1);
    png_build(*L, L->lens + 288, 32, L->dist, L->dcnt, L->dsym, 1);
}

// dynamic Huffman codes (§3.2.7) from bit P: returns the bit after the code lengths, ~0u on error
__device__ __noinline__ uint32_t png_tables_dynamic(PngLds* L, const uint32_t* z, uint32_t lim, uint32_t P) {
    const int lane = threadIdx.x;
    PngBits br;
    br.z = z;
    br.lim = lim;
    br.seek_bit(P);
    const int nlen = (int)br.get(5) + 257, ndist = (int)br.get(5) + 1, ncl = (int)br.get(4) + 4;
    if (nlen > 286 || ndist > 30) return ~0u;
    const uint8_t ord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    __syncthreads();
    if (lane < 19) L->lens[300 + lane] = 0;
    __syncthreads();
    for (int i = 0; i < ncl; ++i) {
        const uint32_t v = br.get(3);
        if (lane == 0) L->lens[300 + ord[i]] = (uint8_t)v;
    }
    __syncthreads();
    if (!png_build(*L, L->lens + 300, 19, L->lit, L->lcnt, L->lsym, 0)) return ~0u;
    int i = 0;
    while (i < nlen + ndist) {
        const int sym = png_decode(br, L->lit, L->lcnt, L->lsym);
        if (sym < 0) return ~0u;
        if (sym < 16) {
            if (lane == 0) L->lens[i] = (uint8_t)sym;
            ++i;
            continue;
        }
        int rep, val = 0;
        if (sym == 16) {
            if (i == 0) return ~0u;
            __syncthreads();
            val = (int)rfl(L->lens[i - 1]);
            rep = 3 + (int)br.get(2);
        } else if (sym == 17) {
            rep = 3 + (int)br.get(3);
        } else {
            rep = 11 + (int)br.get(7);
        }
        if (i + rep > nlen + ndist) return ~0u;
        for (int k = lane; k < rep; k += 64) L->lens[i + k] = (uint8_t)val;
        i += rep;
    }
    __syncthreads();
    if (rfl(L->lens[256]) == 0) return ~0u;                 // no end-of-block code
    // the distance lengths move to lens[288..] so both sets keep their own slots
    const uint8_t dl = lane < ndist ? L->lens[nlen + lane] : 0;
    __syncthreads();
    if (lane < 32) L->lens[288 + lane] = dl;
    __syncthreads();
    if (!png_build(*L, L->lens, nlen, L->lit, L->lcnt, L->lsym, 1) ||
        !png_build(*L, L->lens + 288, ndist, L->dist, L->dcnt, L->dsym, 1))
        return ~0u;
    return (uint32_t)br.consumed();
}

// one token through the bit-serial decoder (a code longer than PNG_FB bits, or an invalid one)
struct PngTok {
    uint32_t P;      // bit after the token
    int sym;         // < 256 literal, 256 end of block, 257 match, -1 invalid
    int len, dist;
};
__device__ __noinline__ PngTok png_serial_token(PngLds* L, const uint32_t* z, uint32_t lim, uint32_t P) {
    PngBits br;
    br.z = z;
    br.lim = lim;
    br.seek_bit(P);
    PngTok t{0, -1, 0, 0};
    const int sy = png_decode(br, L->lit, L->lcnt, L->lsym);
    if (sy >= 0 && sy <= 256) {
        t.sym = sy;
    } else if (sy > 256 && sy - 257 <= 28) {
        const int cc = sy - 257;
        int len;
        if (cc < 8) len = 3 + cc;
        else if (cc == 28) len = 258;
        else {
            const int ebb = (cc - 4) >> 2;
            len = ((4 + (cc & 3)) << ebb) + 3 + (int)br.get(ebb);
        }
        const int dc = png_decode(br, L->dist, L->dcnt, L->dsym);
        if (dc >= 0 && dc <= 29) {
            int d;
            if (dc < 4) d = dc + 1;
            else {
                const int ebb = (dc >> 1) - 1;
                d = ((2 + (dc & 1)) << ebb) + 1 + (int)br.get(ebb);
            }
            t.sym = 257;
            t.len = len;
            t.dist = d;
        }
    }
    t.P = (uint32_t)br.consumed();
    return t;
}

__global__ void __launch_bounds__(64) k_png_inflate(const uint8_t* __restrict__ zbase, const int64_t* __restrict__ offs,
                                                    const PngSegTable* __restrict__ tabs, int H, int W,
                                                    uint8_t* __restrict__ rows, int32_t* __restrict__ status) {
    __shared__ PngLds L;
    const int f = blockIdx.x;
    const int lane = threadIdx.x;
    if (status[f]) return;
    const PngSegTable* T = tabs + f;
    const uint32_t zlen = T->zlen;
    const uint32_t total = (uint32_t)H * (2u * (uint32_t)W + 1u);      // < 2^31 (host check)
    uint8_t* out = rows + (uint64_t)f * png_rstride(H, W);
    const uint32_t* z = reinterpret_cast<const uint32_t*>(zbase + png_zoff(offs[f], f));
    const uint32_t lim = (zlen + 15) / 4;                                // the 16 zero bytes after the stream
    int st = 0;
    uint32_t pos = 0, flushed = 0;
    uint64_t s1 = 0, s2 = 0;
#ifdef PNG_STATS
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    uint64_t n_rounds = 0, n_tok = 0, n_slow = 0, n_match = 0;
#endif

    // zlib header (RFC 1950): CM 8, CINFO <= 7, check bits, no preset dictionary
    uint32_t P = 0;
    {
        const uint32_t cmf = png_bits(z, lim, 0, 8), flg = png_bits(z, lim, 8, 8);
        if ((cmf & 15) != 8 || (cmf >> 4) > 7 || ((cmf << 8) | flg) % 31 != 0 || (flg & 32)) st |= BF_PNG_BAD_ZLIB;
        P = 16;
    }
    bool last = st != 0;
    while (!last) {
        const uint32_t hdr = png_bits(z, lim, P, 3);
        P += 3;
        last = hdr & 1;
        const uint32_t type = hdr >> 1;
        if (type == 0) {                                   // stored
            const uint32_t b = (P + 7) >> 3;
            const uint32_t len = png_bits(z, lim, 8 * b, 16), nlen = png_bits(z, lim, 8 * b + 16, 16);
            if ((len ^ 0xffffu) != nlen) { st |= BF_PNG_BAD_ZLIB; break; }
            if (b + 4 + len > zlen || pos + len > total) { st |= BF_PNG_BAD_ZLIB; break; }
            const uint8_t* zb = reinterpret_cast<const uint8_t*>(z) + b + 4;
            for (uint32_t c = 0; c < len; c += 64 * 16) {
                const uint32_t m = len - c < 64 * 16 ? len - c : 64 * 16;
                for (uint32_t i = lane; i < m; i += 64) L.ring[(pos + i) & (PNG_RING - 1)] = zb[c + i];
                pos += m;
                if (pos - flushed >= PNG_FLUSH) {
                    const uint32_t to = pos & ~15u;
                    png_flush(L, out, flushed, to, total, s1, s2);
                    flushed = to;
                }
                __syncthreads();
            }
            P = 8 * (b + 4 + len);
            continue;
        }
        if (type == 3) { st |= BF_PNG_BAD_ZLIB; break; }
        if (type == 1) {
            png_tables_fixed(&L);
        } else {
            P = rfl(png_tables_dynamic(&L, z, lim, P));      // (a call's result is a VGPR: make it uniform again)
            if (P == ~0u) { st |= BF_PNG_BAD_ZLIB; break; }
        }
        // the block's symbols.  Rounds: lane j decodes the token (literal, or length + distance
        // with their extra bits, or end-of-block) that would start at bit P + j -- every token
        // that can start in the next 64 bits, from one window of 160 bits and two table lookups
        // per lane -- and the scalar unit follows the chain of real token starts from P through
        // the lanes (one readlane per token).  The round's literals are stored by their lanes at
        // once, its matches are copied in stream order by all 64 lanes.  A token whose code is
        // longer than PNG_FB bits (or invalid) ends the round and goes through the bit-serial
        // decoder.
        bool eob = false;
        // the window at P: 64 * PNG_HALVES + 48 bits of candidate tokens (+ 31 of alignment); the
        // next round's is loaded as soon as its P is known, so the scalar loads fly while this round
        // stores its output
        constexpr int NW = 3 + 2 * PNG_HALVES;
        uint32_t Wd[NW];
#pragma unroll
        for (int k = 0; k < NW; ++k) Wd[k] = z[min((P >> 5) + k, lim)];
        while (!eob) {
            // candidate token at bit P + 64 h + lane (half h): literal, length + distance with their
            // extra bits, end of block, or "bit-serial" (a code longer than PNG_FB bits / invalid)
            uint32_t nxt[PNG_HALVES], sz[PNG_HALVES], lit[PNG_HALVES], mlen[PNG_HALVES], dist[PNG_HALVES];
            bool is_lit[PNG_HALVES], is_match[PNG_HALVES];
#pragma unroll
            for (int h = 0; h < PNG_HALVES; ++h) {
                const uint32_t o = (P & 31u) + (uint32_t)lane + 64u * h;
                const uint32_t kk = o >> 5, sh = o & 31u;          // kk in 2h .. 2h + 2
                const uint32_t d0 = kk == 2 * h ? Wd[2 * h] : (kk == 2 * h + 1 ? Wd[2 * h + 1] : Wd[2 * h + 2]);
                const uint32_t d1 = kk == 2 * h ? Wd[2 * h + 1] : (kk == 2 * h + 1 ? Wd[2 * h + 2] : Wd[2 * h + 3]);
                // the first 32 bits at the candidate start (a literal / length code is <= 15 bits)
                const uint32_t b32 = __builtin_amdgcn_alignbit(d1, d0, sh);
                const uint32_t e = L.lit[b32 & ((1u << PNG_FB) - 1u)];
                const uint32_t len1 = e & 15u, sym = e >> 4;
                is_lit[h] = len1 != 0 && sym < 256u;
                const bool is_eob = len1 != 0 && sym == 256u;
                bool mt = false;
                uint32_t T = len1;
                mlen[h] = 0;
                dist[h] = 0;
                // length + distance decode only when some lane of the half decoded a length symbol
                // (literal-heavy streams -- noisy depth -- rarely have one at any of the 64 starts)
                if (__any(len1 != 0 && sym > 256u)) {
                    const uint32_t d2 = kk == 2 * h ? Wd[2 * h + 2] : (kk == 2 * h + 1 ? Wd[2 * h + 3] : Wd[2 * h + 4]);
                    const uint64_t bits = ((uint64_t)__builtin_amdgcn_alignbit(d2, d1, sh) << 32) | b32;
                    const uint32_t c = sym - 257u;                    // length code (257..285)
                    const uint32_t eb = (c < 8u || c == 28u) ? 0u : ((c - 4u) >> 2);
                    const uint32_t base = c < 8u ? 3u + c : (c == 28u ? 258u : ((4u + (c & 3u)) << eb) + 3u);
                    uint64_t b2 = bits >> len1;
                    mlen[h] = base + ((uint32_t)b2 & ((1u << eb) - 1u));
                    b2 >>= eb;
                    const uint32_t e2 = L.dist[(uint32_t)b2 & ((1u << PNG_FB) - 1u)];
                    const uint32_t len2 = e2 & 15u, dsy = e2 >> 4;
                    b2 >>= len2;
                    const uint32_t deb = dsy < 4u ? 0u : (dsy >> 1) - 1u;
                    const uint32_t dbase = dsy < 4u ? dsy + 1u : ((2u + (dsy & 1u)) << deb) + 1u;
                    dist[h] = dbase + ((uint32_t)b2 & ((1u << deb) - 1u));
                    mt = len1 != 0 && sym > 256u && c <= 28u && len2 != 0 && dsy <= 29u;
                    if (mt) T = len1 + eb + len2 + deb;
                }
                is_match[h] = mt;
                // next token start (position 64 h + lane + T), end of block 1024 + start, bit-serial
                // 2048 + position.  The walk stops at the first start >= 64 * PNG_HALVES
                const uint32_t me = 64u * h + (uint32_t)lane;
                nxt[h] = is_lit[h] || mt ? me + T : (is_eob ? 1024u + me + T : 2048u + me);
                sz[h] = is_lit[h] ? 1u : (mt ? mlen[h] : 0u);
                lit[h] = sym;
            }
            // the chain of real token starts (scalar), through the halves in order
            uint32_t at = 0;
            uint64_t mem[PNG_HALVES];
#pragma unroll
            for (int h = 0; h < PNG_HALVES; ++h) mem[h] = 0;
#pragma unroll
            for (int h = 0; h < PNG_HALVES; ++h) {
                while (at < 64u * (h + 1)) {
                    mem[h] |= 1ull << (at - 64u * h);
                    at = __builtin_amdgcn_readlane(nxt[h], at - 64u * h);
                }
            }
            const bool slow = at >= 2048u;
            if (slow) at -= 2048u;
            else if (at >= 1024u) {
                eob = true;
                at -= 1024u;
            }
#ifdef PNG_STATS
            ++n_rounds;
            n_slow += slow;
#pragma unroll
            for (int h = 0; h < PNG_HALVES; ++h) {
                n_tok += __popcll(mem[h]);
                n_match += __popcll(__ballot(((mem[h] >> lane) & 1ull) && is_match[h]));
            }
#endif
            P += at;
            if (!slow) {
#pragma unroll
                for (int k = 0; k < NW; ++k) Wd[k] = z[min((P >> 5) + k, lim)];
            }
            // output offsets of the round's tokens: exclusive scan of their sizes in position order
            uint32_t offv[PNG_HALVES], run = 0;
            bool member[PNG_HALVES];
#pragma unroll
            for (int h = 0; h < PNG_HALVES; ++h) {
                member[h] = (mem[h] >> lane) & 1ull;
                const uint32_t msz = member[h] ? sz[h] : 0u;
                const uint32_t incl = png_wave_scan(msz);
                offv[h] = run + incl - msz;
                run += __builtin_amdgcn_readlane(incl, 63);
            }
            if (run > total - pos) { st |= BF_PNG_SIZE; break; }
#pragma unroll
            for (int h = 0; h < PNG_HALVES; ++h)
                if (member[h] && is_lit[h]) L.ring[(pos + offv[h]) & (PNG_RING - 1)] = (uint8_t)lit[h];
#pragma unroll
            for (int h = 0; h < PNG_HALVES; ++h) {
                uint64_t mm = __ballot(member[h] && is_match[h]);
                while (mm) {
                    const uint32_t j = (uint32_t)__builtin_ctzll(mm);
                    mm &= mm - 1;
                    const uint32_t len = __builtin_amdgcn_readlane(mlen[h], j);
                    const uint32_t d = __builtin_amdgcn_readlane(dist[h], j);
                    const uint32_t dst = pos + __builtin_amdgcn_readlane(offv[h], j);
                    if (d > dst) { st |= BF_PNG_BAD_ZLIB; break; }
                    for (uint32_t k = (uint32_t)lane; k < len; k += 64) {
                        const uint32_t oo = d >= len ? k : k % d;
                        L.ring[(dst + k) & (PNG_RING - 1)] = L.ring[(dst - d + oo) & (PNG_RING - 1)];
                    }
                }
            }
            if (st) break;
            pos += run;
            if (slow) {
                __syncthreads();
                PngTok t = png_serial_token(&L, z, lim, P);
                t.P = rfl(t.P);
                t.sym = (int)rfl((uint32_t)t.sym);
                t.len = (int)rfl((uint32_t)t.len);
                t.dist = (int)rfl((uint32_t)t.dist);
                if (t.sym < 0) { st |= BF_PNG_BAD_ZLIB; break; }
                if (t.sym < 256) {
                    if (pos >= total) { st |= BF_PNG_SIZE; break; }
                    if (lane == 0) L.ring[pos & (PNG_RING - 1)] = (uint8_t)t.sym;
                    ++pos;
                } else if (t.sym == 256) {
                    eob = true;
                } else {
                    const uint32_t len = (uint32_t)t.len, d = (uint32_t)t.dist;
                    if (d > pos) { st |= BF_PNG_BAD_ZLIB; break; }
                    if (len > total - pos) { st |= BF_PNG_SIZE; break; }
                    __syncthreads();
                    for (uint32_t k = lane; k < len; k += 64) {
                        const uint32_t oo = d >= len ? k : k % d;
                        L.ring[(pos + k) & (PNG_RING - 1)] = L.ring[(pos - d + oo) & (PNG_RING - 1)];
                    }
                    pos += len;
                }
                P = t.P;
#pragma unroll
                for (int k = 0; k < NW; ++k) Wd[k] = z[min((P >> 5) + k, lim)];
            }
            if (pos - flushed >= PNG_FLUSH) {
                const uint32_t to = pos & ~15u;
                png_flush(L, out, flushed, to, total, s1, s2);
                flushed = to;
            }
        }
        if (st) break;
        __syncthreads();
    }
    if (!st) {
        png_flush(L, out, flushed, pos, total, s1, s2);
        if (pos != total) st |= BF_PNG_SIZE;
        // Adler-32 (RFC 1950 §8.2): A = 1 + sum d_i, B = n + n * sum d_i - sum i d_i (mod 65521)
        const uint64_t S1 = (uint64_t)bf_wave_sum_i64((long long)s1);
        const uint64_t S2 = (uint64_t)bf_wave_sum_i64((long long)s2);
        const uint64_t M = 65521;
        const uint64_t A = (1 + S1) % M;
        const uint64_t B = ((uint64_t)pos % M + ((uint64_t)pos % M) * (S1 % M) % M + M - S2 % M) % M;
        const uint32_t b = (P + 7) >> 3;
        uint32_t want = 0;
        for (int k = 0; k < 4; ++k) want = (want << 8) | png_bits(z, lim, 8 * (b + k), 8);
        if (b + 4 > zlen || want != (uint32_t)((B << 16) | A)) st |= BF_PNG_BAD_ADLER;
    }
    if (lane == 0 && st) status[f] = st;
#ifdef PNG_STATS
    const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0 && f < 4096) {
        unsigned long long* o = png_stats + f * PNG_NSTAT;
        o[0] = c1 - c0; o[1] = r1 - r0; o[2] = n_rounds; o[3] = n_tok; o[4] = n_slow; o[5] = n_match;
    }
#endif
}

// ---- unfilter (PNG 1.2 §6, bpp = 2) ---------------------------------------------------------
__device__ __forceinline__ uint32_t png_paeth(uint32_t a, uint32_t b, uint32_t c) {
    const int p = (int)a + (int)b - (int)c;
    const int pa = abs(p - (int)a), pb = abs(p - (int)b), pc = abs(p - (int)c);
    return (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
}

// branch-free: every candidate computed, the row's filter type selects by masks (a divergent
// switch became jumps to far blocks, several per step of the unfilter's serial chain)
__device__ __forceinline__ uint32_t png_sel(bool c, uint32_t x, uint32_t y) { return y ^ ((x ^ y) & (0u - (uint32_t)c)); }
__device__ __forceinline__ uint32_t png_pred(uint32_t ft, uint32_t a, uint32_t b, uint32_t c) {
    const int p = (int)a + (int)b - (int)c;
    const int pa = abs(p - (int)a), pb = abs(p - (int)b), pc = abs(p - (int)c);
    const uint32_t pth = png_sel(pa <= pb && pa <= pc, a, png_sel(pb <= pc, b, c));
    uint32_t r = png_sel(ft == 1, a, 0u);
    r = png_sel(ft == 2, b, r);
    r = png_sel(ft == 3, (a + b) >> 1, r);
    return png_sel(ft == 4, pth, r);
}

// OutT uint16_t: the samples (cv2.imread IMREAD_UNCHANGED); float: sample / depth_scale in IEEE
// f32 division (capture_stream.py:203, depth_data.astype(np.float32) / self.depth_scale)
template <typename OutT>
__global__ void __launch_bounds__(64) k_png_unfilter(const uint8_t* __restrict__ rows, int H, int W, float depth_scale,
                                                     OutT* __restrict__ out, int32_t* __restrict__ status) {
    __shared__ uint16_t prev[4096];      // the last row of the previous band (lane 63's outputs)
    const int f = blockIdx.x;
    const int lane = threadIdx.x;
    if (status[f]) return;
    const uint64_t S = 2 * (uint64_t)W + 1;
#ifdef PNG_STATS
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#endif
    const uint8_t* src = rows + (uint64_t)f * png_rstride(H, W);
    OutT* dst = out + (uint64_t)f * H * W;
    int bad = 0;
    for (int b0 = 0; b0 < H; b0 += 64) {
        const int r = b0 + lane;
        const bool valid = r < H;
        const uint8_t* row = src + (uint64_t)(valid ? r : 0) * S;
        const uint32_t ft = valid ? row[0] : 0u;
        bad |= ft > 4;
        uint32_t mine = 0, up_prev = 0;          // (hi << 8 | lo) of this lane's last pixel / last row-above pixel
        // the filtered pixels of a chunk of 8 steps are loaded one chunk ahead
        // every lane loads every step (address clamped into the row, the value selected after), so
        // the 8 loads of a chunk issue back to back instead of one branch and wait each
        auto ld = [&](int x) -> uint32_t {
            const int xc = x < 0 ? 0 : (x >= W ? W - 1 : x);
            // the sample's two bytes as one (unaligned: rows are 2W + 1 bytes) 16-bit load, byte-swapped at use
            return (uint32_t)*reinterpret_cast<const uint16_t*>(row + 1 + 2 * xc);
        };
        // the raw loads go through an empty asm at their use (the next chunk), so the compiler
        // can neither sink them into a branch nor wait for them early
        auto fix = [&](uint32_t (&v)[8], int x0) {
            asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]),
                         "+v"(v[7]));
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int x = x0 + j;
                v[j] = (valid && x >= 0 && x < W) ? (((v[j] & 255u) << 8) | (v[j] >> 8)) : 0u;
            }
        };
        uint32_t cur[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) cur[j] = ld(j - lane);
        fix(cur, -lane);
        for (int t0 = 0; t0 < W + 63; t0 += 8) {
            uint32_t nxt[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) nxt[j] = ld(t0 + 8 + j - lane);     // fixed up next chunk
            // lane 0's row above for the chunk (the previous band's last row), read ahead of the chain
            uint32_t pv[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) pv[j] = prev[t0 + j < W ? t0 + j : 0];
            asm volatile("" : "+v"(pv[0]), "+v"(pv[1]), "+v"(pv[2]), "+v"(pv[3]), "+v"(pv[4]), "+v"(pv[5]),
                         "+v"(pv[6]), "+v"(pv[7]));
#pragma unroll
            for (int j = 0; j < 8; ++j) pv[j] = (b0 > 0 && t0 + j < W) ? pv[j] : 0u;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int x = t0 + j - lane;
                const bool act = valid && x >= 0 && x < W;
                // the row above = lane - 1's pixel of the previous step: a one-lane shift (DPP wave_shr:1)
                const uint32_t nb = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mine, 0x138, 0xf, 0xf, true);
                const uint32_t up = lane == 0 ? pv[j] : nb;
                const uint32_t left = x > 0 ? mine : 0u;
                const uint32_t ul = x > 0 ? up_prev : 0u;
                uint32_t o = 0;
                if (act) {
                    const uint32_t hi = ((cur[j] >> 8) + png_pred(ft, left >> 8, up >> 8, ul >> 8)) & 255u;
                    const uint32_t lo = ((cur[j] & 255u) + png_pred(ft, left & 255u, up & 255u, ul & 255u)) & 255u;
                    o = (hi << 8) | lo;
                    if constexpr (sizeof(OutT) == 2) dst[(uint64_t)r * W + x] = (OutT)o;
                    else dst[(uint64_t)r * W + x] = (float)o / depth_scale;
                    if (lane == 63) prev[x] = (uint16_t)o;
                }
                mine = o;
                up_prev = up;
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) cur[j] = nxt[j];
            fix(cur, t0 + 8 - lane);
        }
        __syncthreads();
    }
    if (__any(bad) && lane == 0) status[f] |= BF_PNG_BAD_FILTER;
#ifdef PNG_STATS
    const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0 && f < 4096) {
        png_stats[f * PNG_NSTAT + 6] = c1 - c0;
        png_stats[f * PNG_NSTAT + 7] = r1 - r0;
    }
#endif
}

BF_API size_t bf_png_workspace_bytes(int F, int H, int W, long long total_file_bytes) {
    if (F < 0 || H <= 0 || W <= 0 || total_file_bytes < 0) return 0;
    return png_tab_bytes(F) + png_list_bytes(F, total_file_bytes) + png_z_bytes(F, total_file_bytes) +
           png_align((size_t)F * png_rstride(H, W) + 16, 256);
}

template <typename OutT>
static int png_decode(const uint8_t* files, const int64_t* offsets, int F, int H, int W, long long total_file_bytes,
                      long long max_file_bytes, float depth_scale, OutT* out, void* work, size_t work_bytes,
                      int32_t* status, void* stream) {
    if (!files || !offsets || !out || !work || !status || F < 0 || H <= 0 || W <= 0 || total_file_bytes < 0 ||
        max_file_bytes < 0 || !(depth_scale > 0.f))
        return BF_ERR_ARG;
    if (W > 4096 || (uint64_t)H * (2 * (uint64_t)W + 1) >= (1ull << 31) || max_file_bytes >= (1ll << 31))
        return BF_ERR_UNSUPPORTED;
    if (work_bytes < bf_png_workspace_bytes(F, H, W, total_file_bytes)) return BF_ERR_CAPACITY;
    if (F == 0) return BF_OK;
    uint8_t* w = static_cast<uint8_t*>(work);
    PngSegTable* tabs = reinterpret_cast<PngSegTable*>(w);
    PngSeg* segs = reinterpret_cast<PngSeg*>(w + png_tab_bytes(F));
    uint8_t* z = w + png_tab_bytes(F) + png_list_bytes(F, total_file_bytes);
    uint8_t* rows = z + png_z_bytes(F, total_file_bytes);
    hipStream_t s = bf_stream(stream);
    hipLaunchKernelGGL(k_png_parse, dim3(F), dim3(64), 0, s, files, offsets, F, H, W, tabs, segs, status);
    const unsigned gx = (unsigned)((max_file_bytes + 16 + 256 * 16 - 1) / (256 * 16));
    hipLaunchKernelGGL(k_png_gather, dim3(gx ? gx : 1, F), dim3(256), 0, s, files, offsets, tabs, segs, z);
    hipLaunchKernelGGL(k_png_inflate, dim3(F), dim3(64), 0, s, z, offsets, tabs, H, W, rows, status);
    hipLaunchKernelGGL(k_png_unfilter<OutT>, dim3(F), dim3(64), 0, s, rows, H, W, depth_scale, out, status);
    return bf_check_launch();
}

BF_API int bf_png_decode_u16(const uint8_t* files, const int64_t* offsets, int F, int H, int W,
                             long long total_file_bytes, long long max_file_bytes, uint16_t* out, void* work,
                             size_t work_bytes, int32_t* status, void* stream) {
    return png_decode(files, offsets, F, H, W, total_file_bytes, max_file_bytes, 1.f, out, work, work_bytes, status,
                      stream);
}

BF_API int bf_png_decode_depth(const uint8_t* files, const int64_t* offsets, int F, int H, int W,
                               long long total_file_bytes, long long max_file_bytes, float depth_scale,
                               float* depth_out, void* work, size_t work_bytes, int32_t* status, void* stream) {
    return png_decode(files, offsets, F, H, W, total_file_bytes, max_file_bytes, depth_scale, depth_out, work,
                      work_bytes, status, stream);
}
