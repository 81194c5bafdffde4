// Datatype pack/unpack for device buffers (gfx950).
//
// The reference walks opt_desc on the host and issues one memcpy — for
// device memory one cuMemcpy — per contiguous run (opal_datatype_pack.h:
// 37-206, opal_datatype_cuda.c:121-145).  Here a datatype becomes a small
// device program of {count, blocklen, stride, disp} elements (the shape of
// opal's ddt_elem_desc, opal_datatype_internal.h:157-164) staged in LDS, and
// one launch moves a whole convertor window: every lane owns G-byte
// granules of the packed stream (G = the widest power of two <= 16 that
// divides every run, displacement and stride, so a granule never crosses a
// run), maps its stream position to the typed address with two integer
// divisions, and copies G bytes.  Packed-side accesses are contiguous across
// lanes (coalesced dwordx4 at G = 16); typed-side accesses are as contiguous
// as the datatype allows.  HBM-bound: 2 x packed bytes of algorithmic
// traffic.  A window that starts or ends off the granule grid is handled
// with byte granules for its unaligned head and tail.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/ompi_amd_ddt.h"
#include "ddt_device.h"
#include "runtime.h"

namespace ompi_amd {

// One convertor window [start, start + head + ngran*G + tail) of the packed
// stream: a G-granule body plus byte-granule head/tail (when the window
// starts or ends off the granule grid), all in ONE launch.
struct ddt_window {
    int64_t start;   // stream position of contiguous byte 0
    int64_t body0;   // first body position (multiple of G)
    int64_t ngran;   // body granules
    int64_t head;    // bytes [start, start + head)
    int64_t tail0;   // tail bytes [tail0, tail0 + tail)
    int64_t tail;
};

template <bool UNPACK>
__device__ __forceinline__ void move_byte(const ddt_elem *el, const ddt_desc &d, const char *src,
                                          char *dst, int64_t p, int64_t start) {
    const int64_t t = typed_offset<uint64_t>(el, d.nelem, (uint64_t)d.size, d.extent, (uint64_t)p);
    if (!UNPACK) dst[p - start] = src[t];
    else dst[t] = src[p - start];
}

// UNPACK = false: contig[p - start] = typed[p];  true: typed[p] = contig[p - start].
// I = uint32_t: fast-division path (stream position / G < 2^32).
template <int G, bool UNPACK, typename I>
__device__ __forceinline__ void ddt_body(const ddt_desc &d, const ddt_elem *el, int nelem, const char *src,
                                         char *dst, const ddt_window &w) {
    using T = typename granule<G>::t;
    constexpr int U = kDdtUnroll;
    const int64_t stride = (int64_t)gridDim.x * kDdtThreads;
    // U granules per lane per pass, lane-contiguous for each u: all U
    // typed addresses first, then U loads in flight, then U stores
    for (int64_t j0 = (int64_t)blockIdx.x * kDdtThreads + threadIdx.x; j0 < w.ngran;
         j0 += stride * U) {
        int64_t toff[U];
        T v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = j0 + u * stride;
            const int64_t p = w.body0 + j * G;
            if (j < w.ngran) {
                if constexpr (sizeof(I) == 4)
                    toff[u] = typed_offset_fast<G>(el, nelem, (uint32_t)(d.size / G), d.sdiv,
                                                   d.extent, (uint32_t)(p / G));
                else
                    toff[u] = typed_offset<I>(el, nelem, (I)d.size, d.extent, (I)p);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = j0 + u * stride;
            const int64_t c = w.body0 + j * G - w.start;  // offset in the contiguous buffer
            if (j < w.ngran)
                v[u] = UNPACK ? *reinterpret_cast<const T *>(src + c)
                              : *reinterpret_cast<const T *>(src + toff[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = j0 + u * stride;
            const int64_t c = w.body0 + j * G - w.start;
            if (j < w.ngran) {
                if (UNPACK) *reinterpret_cast<T *>(dst + toff[u]) = v[u];
                else *reinterpret_cast<T *>(dst + c) = v[u];
            }
        }
    }
    if (blockIdx.x == gridDim.x - 1) {
        for (int64_t k = threadIdx.x; k < w.head + w.tail; k += kDdtThreads) {
            const int64_t p = k < w.head ? w.start + k : w.tail0 + (k - w.head);
            const int64_t t = typed_offset<uint64_t>(el, nelem, (uint64_t)d.size, d.extent, (uint64_t)p);
            if (!UNPACK) dst[p - w.start] = src[t];
            else dst[t] = src[p - w.start];
        }
    }
}

// The element table's address space is known at every read (a table that
// may live in LDS or global memory makes every read a flat load — five per
// granule — as osc_ipc.hip's ddt_acc_kernel measured): one element in
// registers (nelem a constant 1), up to kDdtLdsElems in LDS, else global.
template <int G, bool UNPACK, typename I>
__global__ __launch_bounds__(kDdtThreads) void ddt_kernel(ddt_desc d, const char *src, char *dst,
                                                          ddt_window w) {
    __shared__ ddt_elem lds[kDdtLdsElems];
    if (d.nelem == 1) {
        const ddt_elem e0 = d.elems[0];
        ddt_body<G, UNPACK, I>(d, &e0, 1, src, dst, w);
    } else if (d.nelem <= kDdtLdsElems) {
        for (int i = threadIdx.x; i < d.nelem; i += kDdtThreads) lds[i] = d.elems[i];
        __syncthreads();
        ddt_body<G, UNPACK, I>(d, lds, d.nelem, src, dst, w);
    } else {
        ddt_body<G, UNPACK, I>(d, d.elems, d.nelem, src, dst, w);
    }
}

// Single-element datatypes (every vector / contiguous-of-runs type, the
// common case): positions advance by a constant stride S granules per pass,
// so each lane decomposes its first position once (el, k, w) with divisions
// and then walks by constant increments with one carry per level — no
// division in the loop.  position = el*size + disp + k*stride + w (granules
// of G bytes within a run of blen bytes).
struct ddt_walk {
    int64_t count, bg, stride, disp, extent;  // bg = blen / G
    int64_t size_g;                            // count * bg
};

struct ddt_step {
    int64_t el, k, w;  // a constant advance of the walk, split like a position
};
__device__ __forceinline__ ddt_step walk_split(const ddt_walk &v, int64_t D) {
    const int64_t q = D % v.size_g;
    return {D / v.size_g, q / v.bg, q % v.bg};
}
__device__ __forceinline__ void walk_adv(const ddt_walk &v, int64_t &el, int64_t &k, int64_t &w,
                                         const ddt_step &d) {
    w += d.w;
    k += d.k;
    if (w >= v.bg) { w -= v.bg; ++k; }
    if (k >= v.count) { k -= v.count; ++el; }
    el += d.el;
}

// 16-B granules: chunked persistent shape (the xfer kernels'): workgroup b
// moves chunks b, b + grid, ... of 256 x kVecChunkU packed granules, lane t
// granules t, t + 256, ... of each, non-temporal on both sides.  The walk
// advances by two constants (+256 granules inside a chunk, to the next chunk
// after its last).  Vector of 64-double runs at stride 128
// (tools/ddt_vec_probe.hip, profiles/r05_ddt_vec_probe*.jsonl), one-pass
// shape below -> chunked at 2048 workgroups: 0.640 -> 0.758 of 8 TB/s at
// 256 MiB packed, 0.619 -> 0.721 at 1 GiB (out of the Infinity Cache);
// 2-KiB runs 0.623 -> 0.694 at 1 GiB (512 workgroups: 0.609).
constexpr int kVecChunkU = 4;
constexpr int kVecChunkGrid = 2048;

template <bool UNPACK>
__device__ __forceinline__ void ddt_vec16_body(const ddt_walk &v, const char *src, char *dst,
                                               const ddt_window &w) {
    using T = typename granule<16>::t;
    constexpr int U = kVecChunkU;
    constexpr int64_t C = (int64_t)kDdtThreads * U;
    int64_t j = (int64_t)blockIdx.x * C + threadIdx.x;
    if (j >= w.ngran) return;
    const ddt_step d1 = walk_split(v, kDdtThreads);
    const ddt_step d2 = walk_split(v, (int64_t)gridDim.x * C - (int64_t)(U - 1) * kDdtThreads);
    const int64_t pg0 = w.body0 / 16 + j;
    int64_t el = pg0 / v.size_g;
    const int64_t q = pg0 - el * v.size_g;
    int64_t k = q / v.bg;
    int64_t ww = q - k * v.bg;
    for (; j < w.ngran; j += (int64_t)gridDim.x * C) {
        int64_t toff[U];
        T val[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            toff[u] = el * v.extent + v.disp + k * v.stride + ww * 16;
            if (u + 1 < U) walk_adv(v, el, k, ww, d1);
        }
        walk_adv(v, el, k, ww, d2);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t jj = j + (int64_t)u * kDdtThreads;
            const int64_t c = w.body0 + jj * 16 - w.start;
            if (jj < w.ngran)
                val[u] = __builtin_nontemporal_load(
                    reinterpret_cast<const T *>(UNPACK ? src + c : src + toff[u]));
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t jj = j + (int64_t)u * kDdtThreads;
            const int64_t c = w.body0 + jj * 16 - w.start;
            if (jj < w.ngran)
                __builtin_nontemporal_store(val[u], reinterpret_cast<T *>(UNPACK ? dst + toff[u] : dst + c));
        }
    }
}

template <int G, bool UNPACK>
__global__ __launch_bounds__(kDdtThreads) void ddt_vec_kernel(ddt_walk v, const char *src,
                                                              char *dst, ddt_window w) {
    if constexpr (G == 16) {
        ddt_vec16_body<UNPACK>(v, src, dst, w);
        return;
    }
    using T = typename granule<G>::t;
    constexpr int U = kDdtUnroll;
    const int64_t S = (int64_t)gridDim.x * kDdtThreads;  // granules per step
    const int64_t S_el = S / v.size_g, S_q = S % v.size_g;
    const int64_t S_k = S_q / v.bg, S_w = S_q % v.bg;
    const int64_t j0 = (int64_t)blockIdx.x * kDdtThreads + threadIdx.x;
    if (j0 < w.ngran) {
        const int64_t pg0 = w.body0 / G + j0;
        int64_t el = pg0 / v.size_g;
        const int64_t q = pg0 - el * v.size_g;
        int64_t k = q / v.bg;
        int64_t ww = q - k * v.bg;
        for (int64_t j = j0; j < w.ngran; j += S * U) {
            int64_t toff[U];
            T val[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                toff[u] = el * v.extent + v.disp + k * v.stride + ww * G;
                ww += S_w;
                k += S_k;
                if (ww >= v.bg) { ww -= v.bg; ++k; }
                if (k >= v.count) { k -= v.count; ++el; }
                el += S_el;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t jj = j + u * S;
                const int64_t c = w.body0 + jj * G - w.start;
                if (jj < w.ngran)
                    val[u] = UNPACK ? *reinterpret_cast<const T *>(src + c)
                                    : *reinterpret_cast<const T *>(src + toff[u]);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t jj = j + u * S;
                const int64_t c = w.body0 + jj * G - w.start;
                if (jj < w.ngran) {
                    if (UNPACK) *reinterpret_cast<T *>(dst + toff[u]) = val[u];
                    else *reinterpret_cast<T *>(dst + c) = val[u];
                }
            }
        }
    }
}

// byte head/tail of a single-element window (tiny; generic mapping)
template <bool UNPACK>
__global__ void ddt_vec_edges(ddt_desc d, const char *src, char *dst, ddt_window w) {
    for (int64_t k = threadIdx.x; k < w.head + w.tail; k += blockDim.x) {
        const int64_t p = k < w.head ? w.start + k : w.tail0 + (k - w.head);
        move_byte<UNPACK>(d.elems, d, src, dst, p, w.start);
    }
}


// Staged pack for periodic layouts (the LDS staging of strided gathers).
// The packed stream is a sequence of periods — one datatype instance, or one
// run of a single-run-per-instance vector — of `psize` packed bytes each;
// period j's bytes live at typed + base + j * pext + map[q] (q = byte in the
// period; map = identity for a run).  A workgroup loads the typed span of
// `nper` consecutive periods into LDS with 16-B nt loads (gaps included: the
// dispatcher only takes layouts whose gaps are small enough that HBM fetches
// those sectors anyway), then assembles 16-B packed chunks from LDS at the
// type's granule and stores them with one dwordx4 each.  Sub-16-B runs
// (struct{int,double}, blacs indexed, vector of single doubles) thus move
// with 16-B global accesses on both sides instead of 4- or 8-B granules.
struct iov_job {
    int64_t start, len;
    char *contig;
};

struct ddt_period {
    int64_t psize;      // packed bytes per period
    int64_t pext;       // typed bytes between consecutive periods
    int64_t base;       // typed offset of period 0's lowest byte
    int64_t span;       // typed bytes from a period's lowest byte past its highest
    int64_t nper;       // periods per tile
    int64_t map_bytes;  // LDS bytes holding the map (0: identity)
    const uint16_t *map;  // psize entries: typed offset - lowest, per packed byte
    int64_t nt;         // unpack: typed-side stores non-temporal
};

// Stage 16-B vectors [0, nv) of src into LDS (lane t: t, t + 256, ...),
// kStageBatch loads in flight per lane before any LDS write — a plain
// load -> ds_write loop waits for every load before the next (one 16-B
// load in flight per lane: latency-bound).  need(v) = false skips a vector.
constexpr int kStageBatch = 4;
template <typename NEED>
__device__ __forceinline__ void stage_lds(char *lds, const char *src, int64_t nv, NEED need) {
    typedef unsigned int v4 __attribute__((ext_vector_type(4)));
    const v4 *s = reinterpret_cast<const v4 *>(src);
    v4 *d = reinterpret_cast<v4 *>(lds);
    for (int64_t v0 = threadIdx.x; v0 < nv; v0 += (int64_t)kDdtThreads * kStageBatch) {
        v4 r[kStageBatch];
        bool ok[kStageBatch];
#pragma unroll
        for (int u = 0; u < kStageBatch; ++u) {
            const int64_t v = v0 + (int64_t)u * kDdtThreads;
            ok[u] = v < nv && need(v);
            if (ok[u]) r[u] = __builtin_nontemporal_load(s + v);
        }
#pragma unroll
        for (int u = 0; u < kStageBatch; ++u)
            if (ok[u]) d[v0 + (int64_t)u * kDdtThreads] = r[u];
    }
}

// Tiles tile0, tile0 + tstep, ... of the periods [j0, j1) of one window
// (contig = the window's first packed byte, stream position start); the map
// is staged in LDS by the caller.
template <int G, bool IDENT>
__device__ __forceinline__ void pack_tiles(const ddt_period &P, const char *typed, char *contig,
                                           int64_t start, int64_t j0, int64_t j1, int64_t tile0,
                                           int64_t tstep, const uint16_t *map, char *data) {
    using T = typename granule<G>::t;
    typedef unsigned int v4 __attribute__((ext_vector_type(4)));
    const int t = threadIdx.x;
    constexpr int64_t step = 16 * kDdtThreads;  // packed bytes per lane pass
    const int64_t st_j = step / P.psize, st_q = step % P.psize;
    for (int64_t tile = tile0;; tile += tstep) {
        const int64_t jt = j0 + tile * P.nper;
        if (jt >= j1) break;
        const int64_t nj = min(P.nper, j1 - jt);
        const char *t0 = typed + P.base + jt * P.pext;
        const uintptr_t a0 = (uintptr_t)t0 & ~(uintptr_t)15;
        const uintptr_t a1 = ((uintptr_t)(t0 + (nj - 1) * P.pext + P.span) + 15) & ~(uintptr_t)15;
        const int64_t nv = (int64_t)(a1 - a0) / 16;
        const int64_t toff = (int64_t)((uintptr_t)t0 - a0);
        __syncthreads();  // map staged / previous tile's LDS reads done
        // the whole span, gaps included: reading only the 16-B vectors that
        // hold run bytes (half-line requests for vector bl8) measured 2.86
        // vs 3.71 TB/s with the loads batched (profiles/r03_ddt_stage_batch.jsonl)
        stage_lds(data, t0 - toff, nv, [](int64_t) { return true; });
        __syncthreads();
        const int64_t len = nj * P.psize;               // packed bytes of this tile
        char *c0 = contig + (jt * P.psize - start);     // its first packed byte
        const uintptr_t A0 = (uintptr_t)c0 & ~(uintptr_t)15;
        const int64_t nch = (int64_t)((((uintptr_t)(c0 + len) + 15) & ~(uintptr_t)15) - A0) / 16;
        int64_t r = (int64_t)(A0 - (uintptr_t)c0) + 16 * (int64_t)t;  // tile-relative offset
        int64_t jj = 0, q = 0;
        bool walk = false;
        for (int64_t ch = t; ch < nch; ch += kDdtThreads, r += step) {
            char *cp = reinterpret_cast<char *>(A0 + 16 * ch);
            if (r >= 0 && r + 16 <= len) {
                if (!walk) {  // one division per lane per tile, then walk
                    jj = r / P.psize;
                    q = r - jj * P.psize;
                    walk = true;
                }
                union { v4 v; T e[16 / G]; } buf;
                int64_t j2 = jj, q2 = q;
#pragma unroll
                for (int g = 0; g < 16 / G; ++g) {
                    const int64_t off = toff + j2 * P.pext + (IDENT ? q2 : (int64_t)map[q2]);
                    buf.e[g] = *reinterpret_cast<const T *>(data + off);
                    q2 += G;
                    if (q2 == P.psize) { q2 = 0; ++j2; }
                }
                __builtin_nontemporal_store(buf.v, reinterpret_cast<v4 *>(cp));
            } else {
                for (int g = 0; g < 16 / G; ++g) {  // tile-edge chunk: in-range granules
                    const int64_t rg = r + g * G;
                    if (rg < 0 || rg >= len) continue;
                    const int64_t jg = rg / P.psize, qg = rg - jg * P.psize;
                    const int64_t off = toff + jg * P.pext + (IDENT ? qg : (int64_t)map[qg]);
                    *reinterpret_cast<T *>(cp + g * G) = *reinterpret_cast<const T *>(data + off);
                }
            }
            if (walk) {
                q += st_q;
                jj += st_j;
                if (q >= P.psize) { q -= P.psize; ++jj; }
            }
        }
    }
}

// LDS: the period's byte map (unless IDENT), then the tile's data
template <bool IDENT>
__device__ __forceinline__ uint16_t *stage_map(const ddt_period &P, char *lds) {
    uint16_t *map = reinterpret_cast<uint16_t *>(lds);
    if (!IDENT)
        for (int64_t i = threadIdx.x; i < P.psize; i += kDdtThreads) map[i] = P.map[i];
    return map;
}

template <int G, bool IDENT>
__global__ __launch_bounds__(kDdtThreads) void ddt_pack_tile_kernel(ddt_period P,
                                                                   const char *typed,
                                                                   char *contig, int64_t start,
                                                                   int64_t j0, int64_t j1) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const uint16_t *map = stage_map<IDENT>(P, lds);
    pack_tiles<G, IDENT>(P, typed, contig, start, j0, j1, blockIdx.x, gridDim.x, map,
                         lds + P.map_bytes);
}

// Staged unpack, the mirror of the tile pack: a workgroup brings the packed
// bytes of `nper` periods into LDS with 16-B nt loads (coalesced on the
// contiguous side), then lane t writes packed granules t, t + 256, … of the
// tile to their typed addresses — adjacent lanes store adjacent granules, so
// each store instruction covers a contiguous typed stretch.  Only the typed
// bytes the datatype owns are written (gaps stay untouched).  Per granule
// the position walks by constant increments (one division per lane per
// tile) instead of the generic kernel's element search + two divisions.
template <int G, bool IDENT>
__device__ __forceinline__ void unpack_tiles(const ddt_period &P, const char *contig, char *typed,
                                             int64_t start, int64_t j0, int64_t j1, int64_t tile0,
                                             int64_t tstep, const uint16_t *map, char *data) {
    using T = typename granule<G>::t;
    const int t = threadIdx.x;
    constexpr int64_t step = (int64_t)G * kDdtThreads;  // packed bytes per lane pass
    const int64_t st_j = step / P.psize, st_q = step % P.psize;
    for (int64_t tile = tile0;; tile += tstep) {
        const int64_t jt = j0 + tile * P.nper;
        if (jt >= j1) break;
        const int64_t nj = min(P.nper, j1 - jt);
        const int64_t len = nj * P.psize;                    // packed bytes of this tile
        const char *c0 = contig + (jt * P.psize - start);    // its first packed byte
        const uintptr_t A0 = (uintptr_t)c0 & ~(uintptr_t)15;
        const int64_t nv = (int64_t)((((uintptr_t)(c0 + len) + 15) & ~(uintptr_t)15) - A0) / 16;
        __syncthreads();  // map staged / previous tile's LDS reads done
        // (c0 minus its phase: the pointer keeps the kernel argument's global
        // address space, so these are global_load, not flat_load)
        stage_lds(data, c0 - ((uintptr_t)c0 & 15), nv, [](int64_t) { return true; });
        __syncthreads();
        const char *src = data + ((uintptr_t)c0 - A0);
        char *t0 = typed + P.base + jt * P.pext;
        int64_t r = (int64_t)t * G;
        if (r >= len) continue;
        int64_t j = r / P.psize, q = r - j * P.psize;
        constexpr int U = 4;  // granules per lane per pass: U independent stores in flight
        for (; r < len; r += U * step) {
            int64_t off[U];
            T v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                off[u] = j * P.pext + (IDENT ? q : (int64_t)map[q]);
                q += st_q;
                j += st_j;
                if (q >= P.psize) { q -= P.psize; ++j; }
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (r + u * step < len) v[u] = *reinterpret_cast<const T *>(src + r + u * step);
            if (P.nt) {
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (r + u * step < len) __builtin_nontemporal_store(v[u], reinterpret_cast<T *>(t0 + off[u]));
            } else {
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (r + u * step < len) *reinterpret_cast<T *>(t0 + off[u]) = v[u];
            }
        }
    }
}

template <int G, bool IDENT>
__global__ __launch_bounds__(kDdtThreads) void ddt_unpack_tile_kernel(ddt_period P,
                                                                     const char *contig,
                                                                     char *typed, int64_t start,
                                                                     int64_t j0, int64_t j1) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const uint16_t *map = stage_map<IDENT>(P, lds);
    unpack_tiles<G, IDENT>(P, contig, typed, start, j0, j1, blockIdx.x, gridDim.x, map,
                           lds + P.map_bytes);
}

// One launch over a whole iovec array (the convertor's fAdvance with
// out_size > 1): job j is stream window [start, start + len) to or from the
// contiguous buffer contig (grid row y = job).  The reference fills an iovec
// array run by run with one memcpy / cuMemcpy each
// (opal_generic_simple_pack, opal_datatype_pack.c:273-356); here every
// granule of every iovec is one lane's work in the same launch, so a PML
// fragment train costs one launch instead of one per fragment.

template <int G, bool UNPACK>
__device__ __forceinline__ void ddt_iov_body(const ddt_desc &d, const ddt_elem *el, int nelem, char *typed,
                                             const iov_job &jb) {
    const int64_t start = jb.start, end = jb.start + jb.len;
    const int64_t body0 = min(end, (start + G - 1) / G * G);
    const int64_t body1 = max(body0, end / G * G);
    const int64_t ngran = (body1 - body0) / G;
    using T = typename granule<G>::t;
    constexpr int U = kDdtUnroll;
    const int64_t stride = (int64_t)gridDim.x * kDdtThreads;
    char *c = jb.contig - start;  // contiguous byte of stream position p: c[p]
    for (int64_t j0 = (int64_t)blockIdx.x * kDdtThreads + threadIdx.x; j0 < ngran; j0 += stride * U) {
        int64_t toff[U];
        T v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = j0 + u * stride;
            if (j < ngran)
                toff[u] = typed_offset<uint64_t>(el, nelem, (uint64_t)d.size, d.extent,
                                                 (uint64_t)(body0 + j * G));
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = j0 + u * stride;
            if (j < ngran)
                v[u] = UNPACK ? *reinterpret_cast<const T *>(c + body0 + j * G)
                              : *reinterpret_cast<const T *>(typed + toff[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = j0 + u * stride;
            if (j < ngran) {
                if (UNPACK) *reinterpret_cast<T *>(typed + toff[u]) = v[u];
                else *reinterpret_cast<T *>(c + body0 + j * G) = v[u];
            }
        }
    }
    if (blockIdx.x == gridDim.x - 1) {  // the window's bytes off the granule grid
        const int64_t head = body0 - start, tail = end - body1;
        for (int64_t k = threadIdx.x; k < head + tail; k += kDdtThreads) {
            const int64_t p = k < head ? start + k : body1 + (k - head);
            const int64_t t = typed_offset<uint64_t>(el, nelem, (uint64_t)d.size, d.extent,
                                                     (uint64_t)p);
            if (UNPACK) typed[t] = c[p];
            else c[p] = typed[t];
        }
    }
}

// element table in registers / LDS / global memory, as ddt_kernel
template <int G, bool UNPACK>
__global__ __launch_bounds__(kDdtThreads) void ddt_iov_kernel(ddt_desc d, char *typed,
                                                              const iov_job *jobs) {
    __shared__ ddt_elem lds[kDdtLdsElems];
    const iov_job jb = jobs[blockIdx.y];
    if (d.nelem == 1) {
        const ddt_elem e0 = d.elems[0];
        ddt_iov_body<G, UNPACK>(d, &e0, 1, typed, jb);
    } else if (d.nelem <= kDdtLdsElems) {
        for (int i = threadIdx.x; i < d.nelem; i += kDdtThreads) lds[i] = d.elems[i];
        __syncthreads();
        ddt_iov_body<G, UNPACK>(d, lds, d.nelem, typed, jb);
    } else {
        ddt_iov_body<G, UNPACK>(d, d.elems, d.nelem, typed, jb);
    }
}

// The staged tile kernels over an iovec array (periodic layouts): grid row
// y = job, x = tiles of that job's whole periods; the last x-block also moves
// the job's partial periods at both ends byte by byte (a 64 KiB PML fragment
// rarely starts or ends on a period boundary).
template <int G, bool IDENT, bool UNPACK>
__global__ __launch_bounds__(kDdtThreads) void ddt_iov_tile_kernel(ddt_period P, ddt_desc d,
                                                                   char *typed,
                                                                   const iov_job *jobs) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const uint16_t *map = stage_map<IDENT>(P, lds);
    const iov_job jb = jobs[blockIdx.y];
    const int64_t start = jb.start, end = jb.start + jb.len;
    const int64_t j0 = (start + P.psize - 1) / P.psize, j1 = end / P.psize;
    if (j1 > j0) {
        if (UNPACK)
            unpack_tiles<G, IDENT>(P, jb.contig, typed, start, j0, j1, blockIdx.x, gridDim.x, map,
                                   lds + P.map_bytes);
        else
            pack_tiles<G, IDENT>(P, typed, jb.contig, start, j0, j1, blockIdx.x, gridDim.x, map,
                                 lds + P.map_bytes);
    }
    if (blockIdx.x == gridDim.x - 1) {
        const int64_t h1 = min(end, j0 * P.psize);     // head [start, h1)
        const int64_t t0 = max(h1, j1 * P.psize);      // tail [t0, end)
        const int64_t head = h1 - start, tail = end - t0;
        for (int64_t k = threadIdx.x; k < head + tail; k += kDdtThreads) {
            const int64_t p = k < head ? start + k : t0 + (k - head);
            if (UNPACK) move_byte<true>(d.elems, d, jb.contig, typed, p, start);
            else move_byte<false>(d.elems, d, typed, jb.contig, p, start);
        }
    }
}

}  // namespace ompi_amd

struct ompi_amd_ddt {
    std::vector<ompi_amd::ddt_elem> host;
    ompi_amd::ddt_elem *dev = nullptr;
    int64_t size = 0;
    int64_t extent = 0;
    int64_t max_blen = 0;
    int gran = 1;  // power of two dividing every blen, disp, stride, extent
    // staged-pack plan for one instance as the period (ddt_pack_tile_kernel)
    bool inst_tile = false;
    int64_t lo = 0, hi = 0;     // lowest / one past highest typed byte of an instance
    uint16_t *dmap = nullptr;   // size entries: typed offset - lo per packed byte
};

namespace ompi_amd {

static int pow2_gran(uint64_t v) {
    int g = 16;
    while (g > 1 && (v % (uint64_t)g) != 0) g >>= 1;
    return g;
}

template <bool UNPACK, typename I>
static hipError_t launch_g(int G, const ddt_desc &d, const char *src, char *dst,
                           const ddt_window &w, hipStream_t s) {
    int64_t blocks = (w.ngran + kDdtThreads * kDdtUnroll - 1) / (kDdtThreads * kDdtUnroll);
    blocks = std::max<int64_t>(1, std::min<int64_t>(blocks, 1 << 20));
    const dim3 grid((unsigned)blocks), block(kDdtThreads);
    switch (G) {
    case 16: hipLaunchKernelGGL((ddt_kernel<16, UNPACK, I>), grid, block, 0, s, d, src, dst, w); break;
    case 8: hipLaunchKernelGGL((ddt_kernel<8, UNPACK, I>), grid, block, 0, s, d, src, dst, w); break;
    case 4: hipLaunchKernelGGL((ddt_kernel<4, UNPACK, I>), grid, block, 0, s, d, src, dst, w); break;
    case 2: hipLaunchKernelGGL((ddt_kernel<2, UNPACK, I>), grid, block, 0, s, d, src, dst, w); break;
    default: hipLaunchKernelGGL((ddt_kernel<1, UNPACK, I>), grid, block, 0, s, d, src, dst, w); break;
    }
    return hipGetLastError();
}

template <bool UNPACK>
static hipError_t launch_vec(int G, const ddt_walk &v, const ddt_desc &d, const char *src,
                             char *dst, const ddt_window &w, hipStream_t s) {
    if (w.ngran > 0) {
        int64_t blocks = (w.ngran + kDdtThreads * kDdtUnroll - 1) / (kDdtThreads * kDdtUnroll);
        blocks = std::max<int64_t>(1, std::min<int64_t>(blocks, 1 << 20));
        if (G == 16)  // chunked persistent grid (ddt_vec16_body)
            blocks = std::max<int64_t>(1, std::min<int64_t>(
                kVecChunkGrid, (w.ngran + kDdtThreads * kVecChunkU - 1) / (kDdtThreads * kVecChunkU)));
        const dim3 grid((unsigned)blocks), block(kDdtThreads);
        switch (G) {
        case 16: hipLaunchKernelGGL((ddt_vec_kernel<16, UNPACK>), grid, block, 0, s, v, src, dst, w); break;
        case 8: hipLaunchKernelGGL((ddt_vec_kernel<8, UNPACK>), grid, block, 0, s, v, src, dst, w); break;
        case 4: hipLaunchKernelGGL((ddt_vec_kernel<4, UNPACK>), grid, block, 0, s, v, src, dst, w); break;
        case 2: hipLaunchKernelGGL((ddt_vec_kernel<2, UNPACK>), grid, block, 0, s, v, src, dst, w); break;
        default: hipLaunchKernelGGL((ddt_vec_kernel<1, UNPACK>), grid, block, 0, s, v, src, dst, w); break;
        }
    }
    if (w.head + w.tail > 0)
        hipLaunchKernelGGL((ddt_vec_edges<UNPACK>), dim3(1), dim3(64), 0, s, d, src, dst, w);
    return hipGetLastError();
}

// Staged tile pack / unpack when the layout is periodic, sub-16-B granular (or
// multi-element) and dense enough.  Returns false when the
// generic / walker kernels should run instead.
constexpr int64_t kTileMaxGap = 128;          // bytes of gap the tile reads through
// Run periods (vector-like layouts), unpack: the tile never touches the
// typed gaps (it reads the packed side and writes runs only), so a gap
// costs nothing but LDS — vector bl64 (512-B runs, 512-B gaps) unpacks at
// 5.10 TB/s through the tile vs 4.06 through the per-granule kernel.  The
// pack keeps kTileMaxGap: it stages the typed span gaps included, so wide
// gaps multiply its reads (bl64 packed slower staged, 3.74 vs 4.00 TB/s,
// profiles/r03_ddt_run_maxgap_ab.jsonl).  OMPI_AMD_DDT_RUN_MAXGAP overrides
// the unpack bound (128 = the round-2 behaviour).
static int64_t run_max_gap() {
    static const int64_t v = [] {
        const char *e = getenv("OMPI_AMD_DDT_RUN_MAXGAP");
        return e ? std::max<int64_t>(0, atoll(e)) : (int64_t)4096;
    }();
    return v;
}
constexpr int64_t kTileDataDefault = 16 << 10;  // LDS data bytes per workgroup (tuned)
constexpr int64_t kTileMinWindow = 256 << 10;   // smaller windows: one generic launch

// Layouts whose granule is already 16 B are staged too (vector bl2 / bl8:
// +28 / +30 %, profiles/r01_ddt_tile_wide.jsonl); OMPI_AMD_DDT_TILE_WIDE=0
// restricts the tile to sub-16-B granules and multi-element types.
static bool tile_wide() {
    static const bool v = !(getenv("OMPI_AMD_DDT_TILE_WIDE") && atoi(getenv("OMPI_AMD_DDT_TILE_WIDE")) == 0);
    return v;
}

static int64_t tile_data_bytes() {
    static const int64_t v = [] {
        const char *e = getenv("OMPI_AMD_DDT_TILE_BYTES");
        const int64_t x = e ? atoll(e) : 0;
        return (x >= 4096 && x <= (60 << 10)) ? x : kTileDataDefault;
    }();
    return v;
}

// Unpack: the typed-side stores of a layout whose runs are all shorter than
// 64 B (every store a partial 64-B segment) go non-temporal.  256 MiB
// packed, one convertor call (profiles/r04_unpack_nt_ab.jsonl): blacs
// indexed 1.36 -> 1.63 TB/s, struct{int,double} 2.62 -> 3.72, vector bl2
// (16-B runs) 1.94 -> 3.07; with 64-B runs (bl8) they cost 8 % (5.1 -> 4.7),
// so longer runs keep plain stores.  OMPI_AMD_DDT_UNPACK_NT=0 / 1 forces.
static bool unpack_nt(int64_t max_run) {
    static const int v = [] {
        const char *e = getenv("OMPI_AMD_DDT_UNPACK_NT");
        return e ? atoi(e) : -1;
    }();
    return v >= 0 ? v != 0 : max_run < 64;
}

// Unpack: typed bytes one tile spans (its LDS holds only the packed bytes
// of those periods); OMPI_AMD_DDT_UNPACK_TILE_BYTES, default the pack's —
// halved for periods of many runs (>= 8 elements): 256 MiB blacs-indexed
// unpack (13 runs of 4-52 B) 1.62 -> 1.97 TB/s at 8 KiB, while
// struct{int,double} (2 runs) and vector layouts (1 run) are faster at
// 16 KiB (profiles/r04_unpack_tile_sweep.jsonl, r04_blacs_sweep_nt.jsonl).
static int64_t unpack_tile_bytes(size_t runs) {
    static const int64_t v = [] {
        const char *e = getenv("OMPI_AMD_DDT_UNPACK_TILE_BYTES");
        const int64_t x = e ? atoll(e) : 0;
        return (x >= 1024 && x <= (1 << 20)) ? x : 0;
    }();
    if (v) return v;
    return runs >= 8 ? std::max<int64_t>(4096, tile_data_bytes() / 2) : tile_data_bytes();
}

static bool tile_off() {
    static const bool v = getenv("OMPI_AMD_DDT_TILE") && atoi(getenv("OMPI_AMD_DDT_TILE")) == 0;
    return v;
}

// The period of the staged tile kernels for this layout (false: not
// periodic enough, or a gap too wide to read through); *lds = dynamic LDS.
static bool tile_period(const ompi_amd_ddt_t *ddt, size_t count, int G, bool unpack,
                        ddt_period *out, bool *ident_out, size_t *lds) {
    if (tile_off()) return false;
    ddt_period P{};
    bool ident = false;
    const ddt_elem &x = ddt->host[0];
    if (ddt->host.size() == 1 && x.count > 1 && (G < 16 || tile_wide()) &&
        (count == 1 || ddt->extent == x.count * x.stride) && x.stride > 0 &&
        x.stride - x.blen <= (unpack ? run_max_gap() : kTileMaxGap) &&
        x.stride <= tile_data_bytes() / 4) {
        ident = true;  // period = one run
        P.psize = x.blen;
        P.pext = x.stride;
        P.base = x.disp;
        P.span = x.blen;
    } else if (ddt->inst_tile && (ddt->host.size() > 1 || G < 16 || tile_wide()) &&
               ddt->hi - ddt->lo <= tile_data_bytes() / 4) {
        P.psize = ddt->size;  // period = one instance
        P.pext = ddt->extent;
        P.base = ddt->lo;
        P.span = ddt->hi - ddt->lo;
        P.map = ddt->dmap;
        P.map_bytes = (P.psize * 2 + 15) & ~(int64_t)15;
    } else {
        return false;
    }
    if (P.pext < 0 || P.psize % G != 0) return false;
    if (unpack && P.psize > P.pext) return false;  // the tile's packed bytes must fit its LDS
    P.nt = unpack && unpack_nt(ident ? P.psize : ddt->max_blen) ? 1 : 0;
    const int64_t tb = unpack ? unpack_tile_bytes(ident ? 1 : ddt->host.size()) : tile_data_bytes();
    P.nper = std::max<int64_t>(1, (tb - P.span) / std::max<int64_t>(P.pext, 1) + 1);
    // LDS: the map, then the tile's typed span (the unpack stages only the
    // packed bytes of its periods, but sizing its LDS to those — more
    // workgroups per CU — measured slower: vector bl64 5.4 -> 4.9 TB/s,
    // profiles/r04_unpack_tile_sweep.jsonl), + 32 for the 16-B phase
    *lds = (size_t)P.map_bytes + (size_t)(((P.nper - 1) * P.pext + P.span + 15) & ~(int64_t)15) + 32;
    *out = P;
    *ident_out = ident;
    return true;
}

template <bool UNPACK>
static bool tile_run(const ompi_amd_ddt_t *ddt, size_t count, int G, char *typed, char *contig,
                     int64_t start, int64_t end, const ddt_desc &d, hipStream_t s,
                     hipError_t *err) {
    if (end - start < kTileMinWindow) return false;
    ddt_period P{};
    bool ident = false;
    size_t lds = 0;
    if (!tile_period(ddt, count, G, UNPACK, &P, &ident, &lds)) return false;
    const int64_t j0 = (start + P.psize - 1) / P.psize, j1 = end / P.psize;
    if (j1 <= j0) return false;
    const int64_t tiles = (j1 - j0 + P.nper - 1) / P.nper;
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(tiles, 2048));
    hipError_t e = hipSuccess;
#define TILE(GG)                                                                               \
    case GG:                                                                                   \
        if (UNPACK && ident)                                                                   \
            hipLaunchKernelGGL((ddt_unpack_tile_kernel<GG, true>), dim3(grid),                 \
                               dim3(kDdtThreads), lds, s, P, contig, typed, start, j0, j1);     \
        else if (UNPACK)                                                                       \
            hipLaunchKernelGGL((ddt_unpack_tile_kernel<GG, false>), dim3(grid),                \
                               dim3(kDdtThreads), lds, s, P, contig, typed, start, j0, j1);     \
        else if (ident)                                                                        \
            hipLaunchKernelGGL((ddt_pack_tile_kernel<GG, true>), dim3(grid), dim3(kDdtThreads), \
                               lds, s, P, typed, contig, start, j0, j1);                        \
        else                                                                                   \
            hipLaunchKernelGGL((ddt_pack_tile_kernel<GG, false>), dim3(grid), dim3(kDdtThreads), \
                               lds, s, P, typed, contig, start, j0, j1);                        \
        break;
    switch (G) {
        TILE(16)
        TILE(8)
        TILE(4)
        TILE(2)
        TILE(1)
    default:
        return false;
    }
#undef TILE
    e = hipGetLastError();
    // partial periods at the window ends: generic byte mapping
    const ddt_window w{start, start, 0, j0 * P.psize - start, j1 * P.psize, end - j1 * P.psize};
    if (e == hipSuccess && w.head + w.tail > 0) {
        hipLaunchKernelGGL((ddt_vec_edges<UNPACK>), dim3(1), dim3(kDdtThreads), 0, s, d,
                           UNPACK ? contig : typed, UNPACK ? typed : contig, w);
        e = hipGetLastError();
    }
    *err = e;
    return true;
}

template <bool UNPACK>
static int ddt_run(const ompi_amd_ddt_t *ddt, size_t count, const void *typed, void *contig,
                   size_t offset, size_t bytes, size_t *done, hipStream_t s) {
    if (!ddt || (!typed && count) || !done) return OMPI_AMD_ERR_BAD_PARAM;
    const uint64_t total = (uint64_t)ddt->size * count;
    *done = 0;
    if (offset >= total || bytes == 0) return OMPI_AMD_SUCCESS;
    if (bytes > total - offset) bytes = (size_t)(total - offset);
    if (!contig) return OMPI_AMD_ERR_BAD_PARAM;

    ddt_desc d{ddt->dev, (int)ddt->host.size(), ddt->size, ddt->extent, {0u, 0u, 0u}};
    // Granule: divides the type program, the typed base and the contiguous
    // buffer's alignment relative to the stream position.
    const uint64_t contig_skew = (uint64_t)((uintptr_t)contig - (uintptr_t)offset);
    int G = std::min({ddt->gran, pow2_gran((uintptr_t)typed), pow2_gran(contig_skew)});
    const int64_t start = (int64_t)offset, end = (int64_t)(offset + bytes);
    const int64_t body0 = (start + G - 1) / G * G;
    const int64_t body1 = std::max(body0, end / G * G);
    // contiguous buffer is indexed from `offset`: pass base = offset
    const char *tsrc = UNPACK ? (const char *)contig : (const char *)typed;
    char *tdst = UNPACK ? (char *)typed : (char *)contig;
    ddt_window w{start, body0, (body1 - body0) / G, body0 - start, body1, end - body1};
    if (body0 >= end) w = {start, start, 0, end - start, end, 0};
    // 32-bit granule arithmetic when positions, the type size and every
    // blocklen fit in G units
    // multiply-high division measured no faster than the 64-bit divide on
    // MI355X (profiles/r01_ddt_sweep_*fastdiv.jsonl): opt-in only
    static const bool fast_ok = getenv("OMPI_AMD_DDT_FASTDIV") && atoi(getenv("OMPI_AMD_DDT_FASTDIV"));
    const bool fast = fast_ok && total / (uint64_t)G < (1ull << 32) &&
                      (uint64_t)ddt->max_blen / (uint64_t)G < (1ull << 32) &&
                      (uint64_t)ddt->size / (uint64_t)G < (1ull << 32);
    hipError_t e;
    if (tile_run<UNPACK>(ddt, count, G, (char *)typed, (char *)contig, start, end, d, s, &e)) {
        // staged LDS tile pack / unpack (+ generic bytes for partial periods)
    } else if (ddt->host.size() == 1) {
        const ddt_elem &x = ddt->host[0];
        const ddt_walk v{x.count, x.blen / G, x.stride, x.disp, ddt->extent, x.count * (x.blen / G)};
        e = launch_vec<UNPACK>(G, v, d, tsrc, tdst, w, s);
    } else if (fast) {
        d.sdiv = make_fdiv((uint32_t)(ddt->size / G));
        e = launch_g<UNPACK, uint32_t>(G, d, tsrc, tdst, w, s);
    } else {
        e = launch_g<UNPACK, uint64_t>(G, d, tsrc, tdst, w, s);
    }
    if (e != hipSuccess) return record_hip(e, "ddt kernel launch");
    *done = bytes;
    return OMPI_AMD_SUCCESS;
}

// Per-thread job table for ddt_iov: pinned host staging + a device copy,
// reused once the previous call's kernel has read it (event).
struct iov_table {
    iov_job *host = nullptr, *dev = nullptr;
    size_t cap = 0;
    hipEvent_t used = nullptr;  // after the last kernel that read `dev`
    bool pending = false;
};
static thread_local iov_table tls_iov;

static int iov_reserve(size_t n) {
    iov_table &t = tls_iov;
    if (t.pending) {  // the previous launch still reads the table
        const hipError_t e = hipEventSynchronize(t.used);
        if (e != hipSuccess) return record_hip(e, "hipEventSynchronize (iov table)");
        t.pending = false;
    }
    if (!t.used && hipEventCreateWithFlags(&t.used, hipEventDisableTiming) != hipSuccess)
        return record_hip(hipGetLastError(), "hipEventCreate (iov table)");
    if (n <= t.cap) return OMPI_AMD_SUCCESS;
    const size_t want = std::max<size_t>(n, 2 * t.cap);
    if (t.host) hip_ignore(hipHostFree(t.host));
    if (t.dev) hip_ignore(hipFree(t.dev));
    t.host = nullptr;
    t.dev = nullptr;
    t.cap = 0;
    hipError_t e = hipHostMalloc((void **)&t.host, want * sizeof(iov_job), hipHostMallocDefault);
    if (e == hipSuccess) e = hipMalloc((void **)&t.dev, want * sizeof(iov_job));
    if (e != hipSuccess) return record_hip(e, "iov job table");
    t.cap = want;
    return OMPI_AMD_SUCCESS;
}

// The fAdvance contract (convertor_advance_fct_t, opal_convertor.h:64-67;
// opal_generic_simple_pack, opal_datatype_pack.c:273-369): fill (pack) or
// drain (unpack) iov[0 .. *out_size) in order from stream position
// `position`, each entry up to its iov_len; iov_len becomes the bytes used,
// *out_size the entries used (all of them unless the stream ends inside
// one), *max_data the total.  Returns 1 when the stream is complete, 0 when
// data remains, a negative OMPI_AMD_ERR_* on error.  One launch for all
// entries (the single-entry case takes the tuned window kernels).
template <bool UNPACK>
static int ddt_iov(const ompi_amd_ddt_t *ddt, size_t count, void *typed, size_t position,
                   ompi_amd_iovec_t *iov, uint32_t *out_size, size_t *max_data, hipStream_t s) {
    if (!ddt || !out_size || !max_data || (*out_size && !iov) || (!typed && count))
        return OMPI_AMD_ERR_BAD_PARAM;
    const uint64_t total = (uint64_t)ddt->size * count;
    *max_data = 0;
    if (position >= total) {
        *out_size = 0;
        return 1;
    }
    // host pass: assign stream windows to iovecs
    uint64_t pos = position;
    uint32_t used = 0;
    int G = std::min(ddt->gran, pow2_gran((uintptr_t)typed));
    int64_t most = 0;
    for (uint32_t i = 0; i < *out_size && pos < total; ++i) {
        const uint64_t take = std::min<uint64_t>(iov[i].iov_len, total - pos);
        if (take && !iov[i].iov_base) return OMPI_AMD_ERR_BAD_PARAM;
        iov[i].iov_len = (size_t)take;
        if (take) {
            G = std::min(G, pow2_gran((uint64_t)((uintptr_t)iov[i].iov_base - (uintptr_t)pos)));
            most = std::max<int64_t>(most, (int64_t)take);
        }
        pos += take;
        used = i + 1;
    }
    if (pos < total) used = *out_size;
    const uint64_t moved = pos - position;
    int jobs = 0;
    for (uint32_t i = 0; i < used; ++i) jobs += iov[i].iov_len ? 1 : 0;
    if (jobs == 1) {  // one window: the tuned kernels (staged tile, walker)
        for (uint32_t i = 0; i < used; ++i) {
            if (!iov[i].iov_len) continue;
            size_t done = 0;
            const int rc = ddt_run<UNPACK>(ddt, count, typed, iov[i].iov_base, (size_t)position,
                                           iov[i].iov_len, &done, s);
            if (rc != OMPI_AMD_SUCCESS) return rc;
        }
    } else if (jobs > 1) {
        int rc = iov_reserve((size_t)jobs);
        if (rc != OMPI_AMD_SUCCESS) return rc;
        iov_table &t = tls_iov;
        uint64_t p = position;
        int k = 0;
        for (uint32_t i = 0; i < used; ++i) {
            if (iov[i].iov_len) t.host[k++] = {(int64_t)p, (int64_t)iov[i].iov_len, (char *)iov[i].iov_base};
            p += iov[i].iov_len;
        }
        hipError_t e = hipMemcpyAsync(t.dev, t.host, (size_t)jobs * sizeof(iov_job),
                                      hipMemcpyHostToDevice, s);
        const ddt_desc d{ddt->dev, (int)ddt->host.size(), ddt->size, ddt->extent, {0u, 0u, 0u}};
        const int64_t per = (int64_t)kDdtThreads * kDdtUnroll * G;
        const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>((most + per - 1) / per, 1024));
        // periodic layouts: the staged tile kernels per job (LDS-staged
        // 16-B accesses on both sides instead of per-granule searches)
        ddt_period P{};
        bool ident = false;
        size_t lds = 0;
        const bool tiled = tile_period(ddt, count, G, UNPACK, &P, &ident, &lds);
        // whole periods of the longest job, in tiles (+1: a job need not start
        // on a period boundary)
        const unsigned tgx = tiled ? (unsigned)std::max<int64_t>(
                                         1, std::min<int64_t>((most / std::max<int64_t>(P.psize, 1) +
                                                               P.nper) / P.nper, 2048))
                                   : 1u;
        for (int j0 = 0; e == hipSuccess && j0 < jobs; j0 += 65535) {
            const dim3 grid(gx, (unsigned)std::min(65535, jobs - j0));
            const iov_job *tab = t.dev + j0;
            if (tiled) {
                const dim3 tgrid(tgx, grid.y);
#define IOVT(GG)                                                                                \
    case GG:                                                                                    \
        if (ident)                                                                              \
            hipLaunchKernelGGL((ddt_iov_tile_kernel<GG, true, UNPACK>), tgrid, dim3(kDdtThreads), \
                               lds, s, P, d, (char *)typed, tab);                               \
        else                                                                                    \
            hipLaunchKernelGGL((ddt_iov_tile_kernel<GG, false, UNPACK>), tgrid, dim3(kDdtThreads), \
                               lds, s, P, d, (char *)typed, tab);                               \
        break;
                switch (G) {
                    IOVT(16) IOVT(8) IOVT(4) IOVT(2)
                default: IOVT(1)
                }
#undef IOVT
            } else {
                switch (G) {
#define IOVK(GG) case GG: hipLaunchKernelGGL((ddt_iov_kernel<GG, UNPACK>), grid, dim3(kDdtThreads), 0, s, d, (char *)typed, tab); break;
                    IOVK(16) IOVK(8) IOVK(4) IOVK(2)
                default: IOVK(1)
#undef IOVK
                }
            }
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipEventRecord(t.used, s);
        if (e != hipSuccess) return record_hip(e, "ddt iovec launch");
        t.pending = true;
    }
    *out_size = used;
    *max_data = (size_t)moved;
    return pos == total ? 1 : 0;
}

}  // namespace ompi_amd

using namespace ompi_amd;

namespace ompi_amd {
bool ddt_view_of(const ompi_amd_ddt_t *ddt, ddt_view *out) {
    if (!ddt || !ddt->dev || ddt->host.empty() || !out) return false;
    out->d = ddt_desc{ddt->dev, (int)ddt->host.size(), ddt->size, ddt->extent, {0u, 0u, 0u}};
    int64_t lo = INT64_MAX, hi = INT64_MIN;
    for (const auto &e : ddt->host) {
        const int64_t last = (e.count - 1) * e.stride;  // stride may be negative
        lo = std::min(lo, e.disp + std::min<int64_t>(0, last));
        hi = std::max(hi, e.disp + std::max<int64_t>(0, last) + e.blen);
    }
    out->lo = lo;
    out->hi = hi;
    out->gran = ddt->gran;
    out->max_blen = ddt->max_blen;
    return true;
}
}  // namespace ompi_amd

extern "C" {

int ompi_amd_ddt_pack_iov(const ompi_amd_ddt_t *ddt, size_t count, const void *typed,
                          size_t position, ompi_amd_iovec_t *iov, uint32_t *out_size,
                          size_t *max_data, void *stream) {
    return ddt_iov<false>(ddt, count, const_cast<void *>(typed), position, iov, out_size, max_data,
                          as_stream(stream));
}

int ompi_amd_ddt_unpack_iov(const ompi_amd_ddt_t *ddt, size_t count, void *typed,
                            size_t position, ompi_amd_iovec_t *iov, uint32_t *out_size,
                            size_t *max_data, void *stream) {
    return ddt_iov<true>(ddt, count, typed, position, iov, out_size, max_data, as_stream(stream));
}

int ompi_amd_ddt_create_elems(const ompi_amd_ddt_elem_t *elems, int nelems, int64_t extent,
                              ompi_amd_ddt_t **out) {
    if (!out || nelems <= 0 || !elems) return OMPI_AMD_ERR_BAD_PARAM;
    auto *d = new (std::nothrow) ompi_amd_ddt;
    if (!d) return OMPI_AMD_ERR_BAD_PARAM;
    int64_t prefix = 0;
    uint64_t gcd_acc = (uint64_t)(extent < 0 ? -extent : extent);
    for (int i = 0; i < nelems; ++i) {
        const ompi_amd_ddt_elem_t &x = elems[i];
        if (x.count <= 0 || x.blocklen <= 0) {
            delete d;
            return OMPI_AMD_ERR_BAD_PARAM;
        }
        ddt_elem e{x.count, x.blocklen, x.count > 1 ? x.stride : x.blocklen, x.disp, prefix, {}, 0};
        for (int lg = 0; lg < 5; ++lg) {
            const int64_t bg = e.blen >> lg;
            e.bdiv[lg] = ((e.blen & ((1 << lg) - 1)) == 0 && bg < (1ll << 32))
                             ? make_fdiv((uint32_t)bg) : fastdiv{0u, 0u, 0u};
        }
        d->max_blen = std::max(d->max_blen, e.blen);
        prefix += e.count * e.blen;
        gcd_acc |= (uint64_t)e.blen | (uint64_t)(e.disp < 0 ? -e.disp : e.disp) |
                   (uint64_t)(e.stride < 0 ? -e.stride : e.stride);
        d->host.push_back(e);
    }
    d->size = prefix;
    d->extent = extent;
    d->gran = pow2_gran(gcd_acc);
    // Staged-pack plan with one instance as the period: small instances
    // whose runs leave gaps of at most kTileMaxGap bytes (within an
    // instance and between consecutive instances).
    std::vector<uint16_t> imap;
    if (d->size <= 8192) {
        std::vector<std::pair<int64_t, int64_t>> runs;  // [begin, end) typed
        for (const auto &e : d->host)
            for (int64_t k = 0; k < e.count; ++k)
                runs.emplace_back(e.disp + k * e.stride, e.disp + k * e.stride + e.blen);
        int64_t lo = runs[0].first, hi = runs[0].second;
        for (const auto &r : runs) { lo = std::min(lo, r.first); hi = std::max(hi, r.second); }
        std::vector<std::pair<int64_t, int64_t>> sorted = runs;
        std::sort(sorted.begin(), sorted.end());
        int64_t gap = 0, reach = sorted[0].second;
        for (const auto &r : sorted) {
            gap = std::max(gap, r.first - reach);
            reach = std::max(reach, r.second);
        }
        gap = std::max(gap, extent - (hi - lo));
        if (hi - lo < 65536 && gap <= kTileMaxGap && extent > 0) {
            for (const auto &r : runs)
                for (int64_t b = r.first; b < r.second; ++b) imap.push_back((uint16_t)(b - lo));
            d->inst_tile = true;
            d->lo = lo;
            d->hi = hi;
        }
    }
    const size_t nb = d->host.size() * sizeof(ddt_elem);
    hipError_t err = hipMalloc(&d->dev, nb);
    if (err == hipSuccess) err = hipMemcpy(d->dev, d->host.data(), nb, hipMemcpyHostToDevice);
    if (err == hipSuccess && d->inst_tile) {
        err = hipMalloc(&d->dmap, imap.size() * sizeof(uint16_t));
        if (err == hipSuccess)
            err = hipMemcpy(d->dmap, imap.data(), imap.size() * sizeof(uint16_t),
                            hipMemcpyHostToDevice);
    }
    // a copy from pageable memory may return before the bytes reach the
    // device, and the kernels that read the program run on
    // other (non-blocking) streams: wait for the null stream's copies here
    if (err == hipSuccess) err = hipStreamSynchronize(nullptr);
    if (err != hipSuccess) {
        int rc = record_hip(err, "ddt descriptor upload");
        if (d->dev) hip_ignore(hipFree(d->dev));
        if (d->dmap) hip_ignore(hipFree(d->dmap));
        delete d;
        return rc;
    }
    *out = d;
    return OMPI_AMD_SUCCESS;
}

int ompi_amd_ddt_create(const ompi_amd_ddt_block_t *blocks, int nblocks, int64_t extent,
                        ompi_amd_ddt_t **out) {
    if (!out || nblocks <= 0 || !blocks) return OMPI_AMD_ERR_BAD_PARAM;
    // 1) merge runs that touch (disp_i + len_i == disp_{i+1})
    std::vector<ompi_amd_ddt_block_t> runs;
    for (int i = 0; i < nblocks; ++i) {
        if (blocks[i].len <= 0) return OMPI_AMD_ERR_BAD_PARAM;
        if (!runs.empty() && runs.back().disp + runs.back().len == blocks[i].disp)
            runs.back().len += blocks[i].len;
        else
            runs.push_back(blocks[i]);
    }
    // 2) fold equal-length runs at a constant stride into one element
    std::vector<ompi_amd_ddt_elem_t> elems;
    for (size_t i = 0; i < runs.size();) {
        ompi_amd_ddt_elem_t e{1, runs[i].len, runs[i].len, runs[i].disp};
        size_t j = i + 1;
        if (j < runs.size() && runs[j].len == e.blocklen) {
            const int64_t st = runs[j].disp - runs[i].disp;
            while (j < runs.size() && runs[j].len == e.blocklen &&
                   runs[j].disp - runs[j - 1].disp == st) ++j;
            e.count = (int64_t)(j - i);
            e.stride = st;
        }
        elems.push_back(e);
        i = j;
    }
    return ompi_amd_ddt_create_elems(elems.data(), (int)elems.size(), extent, out);
}

int ompi_amd_ddt_destroy(ompi_amd_ddt_t *ddt) {
    if (!ddt) return OMPI_AMD_SUCCESS;
    if (ddt->dev) hip_ignore(hipFree(ddt->dev));
    if (ddt->dmap) hip_ignore(hipFree(ddt->dmap));
    delete ddt;
    return OMPI_AMD_SUCCESS;
}

size_t ompi_amd_ddt_size(const ompi_amd_ddt_t *ddt) { return ddt ? (size_t)ddt->size : 0; }

int ompi_amd_ddt_nelems(const ompi_amd_ddt_t *ddt) { return ddt ? (int)ddt->host.size() : 0; }

int ompi_amd_ddt_pack(const ompi_amd_ddt_t *ddt, size_t count, const void *src, void *dst,
                      size_t offset, size_t bytes, size_t *done, void *stream) {
    return ddt_run<false>(ddt, count, src, dst, offset, bytes, done, as_stream(stream));
}

int ompi_amd_ddt_unpack(const ompi_amd_ddt_t *ddt, size_t count, const void *src, void *dst,
                        size_t offset, size_t bytes, size_t *done, void *stream) {
    return ddt_run<true>(ddt, count, dst, (void *)src, offset, bytes, done, as_stream(stream));
}

}  // extern "C"
