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
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/ompi_amd_ddt.h"
#include "runtime.h"

namespace ompi_amd {

// Division by a launch-invariant 32-bit divisor d as multiply-high + shifts
// (Granlund-Montgomery round-up method): q = (t + ((n - t) >> s1)) >> s2,
// t = umulhi(n, m); d = 1 gives m = 0, s1 = s2 = 0.  Exact for every
// 32-bit n.  Replaces two v_div-style ~40-instruction sequences per granule.
struct fastdiv {
    uint32_t m, s1, s2;
};

static fastdiv make_fdiv(uint32_t d) {
    if (d <= 1) return {0u, 0u, 0u};
    uint32_t l = 0;
    while ((1ull << l) < d) ++l;  // ceil(log2 d)
    const uint64_t m = ((1ull << 32) * ((1ull << l) - d)) / d + 1;
    return {(uint32_t)m, 1u, l - 1};
}

__device__ __forceinline__ uint32_t fdiv_q(uint32_t n, const fastdiv &f) {
    const uint32_t t = __umulhi(n, f.m);
    return (t + ((n - t) >> f.s1)) >> f.s2;
}

struct ddt_elem {
    int64_t count;   // repetitions
    int64_t blen;    // bytes per repetition
    int64_t stride;  // bytes between repetitions
    int64_t disp;    // byte displacement of the first repetition
    int64_t prefix;  // packed bytes of the type before this element
    fastdiv bdiv[5];    // blen / G for G = 1, 2, 4, 8, 16 (when it fits 32 bits)
    uint32_t pad;
};

constexpr int kDdtThreads = 256;
constexpr int kDdtUnroll = 8;
constexpr int kDdtLdsElems = 256;

struct ddt_desc {
    const ddt_elem *elems;  // device copy
    int nelem;
    int64_t size;    // packed bytes per datatype element
    int64_t extent;
    fastdiv sdiv;       // size / G of this launch (fast path only)
};

// Largest i with elems[i].prefix <= q.
__device__ __forceinline__ int find_elem(const ddt_elem *e, int n, int64_t q) {
    if (n <= 8) {
        int i = 0;
        for (int j = 1; j < n; ++j)
            if (e[j].prefix <= q) i = j;
        return i;
    }
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (e[mid].prefix <= q) lo = mid; else hi = mid - 1;
    }
    return lo;
}

template <int G> struct granule;
template <> struct granule<1> { using t = uint8_t; };
template <> struct granule<2> { using t = uint16_t; };
template <> struct granule<4> { using t = uint32_t; };
template <> struct granule<8> { using t = uint64_t; };
template <> struct granule<16> { typedef unsigned int t __attribute__((ext_vector_type(4))); };

// Typed-layout byte address of packed stream position p.
template <typename I>
__device__ __forceinline__ int64_t typed_offset(const ddt_elem *e, int n, I size, int64_t extent,
                                                I p) {
    const I el = p / size;
    const I q = p - el * size;
    const int i = find_elem(e, n, (int64_t)q);
    const I r = q - (I)e[i].prefix;
    const I k = r / (I)e[i].blen;
    const I w = r - k * (I)e[i].blen;
    return (int64_t)el * extent + e[i].disp + (int64_t)k * e[i].stride + (int64_t)w;
}

// Fast path: all quantities in G-granule units fit 32 bits.
template <int G>
__device__ __forceinline__ int64_t typed_offset_fast(const ddt_elem *e, int n, uint32_t size_g,
                                                     const fastdiv &sdiv, int64_t extent,
                                                     uint32_t pg) {
    constexpr int LG = G == 16 ? 4 : G == 8 ? 3 : G == 4 ? 2 : G == 2 ? 1 : 0;
    const uint32_t el = fdiv_q(pg, sdiv);
    const uint32_t q = pg - el * size_g;
    const int i = find_elem(e, n, (int64_t)q << LG);
    const uint32_t r = q - (uint32_t)(e[i].prefix >> LG);
    const uint32_t k = fdiv_q(r, e[i].bdiv[LG]);
    const uint32_t w = r - k * (uint32_t)(e[i].blen >> LG);
    return (int64_t)el * extent + e[i].disp + (int64_t)k * e[i].stride + ((int64_t)w << LG);
}

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
__global__ __launch_bounds__(kDdtThreads) void ddt_kernel(ddt_desc d, const char *src, char *dst,
                                                          ddt_window w) {
    __shared__ ddt_elem lds[kDdtLdsElems];
    const ddt_elem *el = d.elems;
    if (d.nelem <= kDdtLdsElems) {
        for (int i = threadIdx.x; i < d.nelem; i += kDdtThreads) lds[i] = d.elems[i];
        __syncthreads();
        el = lds;
    }
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
                    toff[u] = typed_offset_fast<G>(el, d.nelem, (uint32_t)(d.size / G), d.sdiv,
                                                   d.extent, (uint32_t)(p / G));
                else
                    toff[u] = typed_offset<I>(el, d.nelem, (I)d.size, d.extent, (I)p);
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
            move_byte<UNPACK>(el, d, src, dst, p, w.start);
        }
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

template <int G, bool UNPACK>
__global__ __launch_bounds__(kDdtThreads) void ddt_vec_kernel(ddt_walk v, const char *src,
                                                              char *dst, ddt_window w) {
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

}  // namespace ompi_amd

struct ompi_amd_ddt {
    std::vector<ompi_amd::ddt_elem> host;
    ompi_amd::ddt_elem *dev = nullptr;
    int64_t size = 0;
    int64_t extent = 0;
    int64_t max_blen = 0;
    int gran = 1;  // power of two dividing every blen, disp, stride, extent
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
    if (ddt->host.size() == 1) {
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

}  // namespace ompi_amd

using namespace ompi_amd;

extern "C" {

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
    const size_t nb = d->host.size() * sizeof(ddt_elem);
    hipError_t err = hipMalloc(&d->dev, nb);
    if (err == hipSuccess) err = hipMemcpy(d->dev, d->host.data(), nb, hipMemcpyHostToDevice);
    if (err != hipSuccess) {
        int rc = record_hip(err, "ddt descriptor upload");
        if (d->dev) (void)hipFree(d->dev);
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
    if (ddt->dev) (void)hipFree(ddt->dev);
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
