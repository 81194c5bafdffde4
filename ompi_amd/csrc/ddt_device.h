// Device view of a datatype program (ddt_kernels.hip): the element table,
// the typed-offset mapping of a packed stream position, and the accessor
// other kernels use (osc_ipc.hip's derived-datatype accumulate).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/ompi_amd_ddt.h"

namespace ompi_amd {

// Division by a launch-invariant 32-bit divisor d as multiply-high + shifts
// (Granlund-Montgomery round-up method): q = (t + ((n - t) >> s1)) >> s2,
// t = umulhi(n, m); d = 1 gives m = 0, s1 = s2 = 0.  Exact for every
// 32-bit n.  Replaces two v_div-style ~40-instruction sequences per granule.
struct fastdiv {
    uint32_t m, s1, s2;
};

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

inline fastdiv make_fdiv(uint32_t d) {  // host side
    if (d <= 1) return {0u, 0u, 0u};
    uint32_t l = 0;
    while ((1ull << l) < d) ++l;  // ceil(log2 d)
    const uint64_t m = ((1ull << 32) * ((1ull << l) - d)) / d + 1;
    return {(uint32_t)m, 1u, l - 1};
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

// A program as other translation units see it (ddt_view_of).
struct ddt_view {
    ddt_desc d;
    int64_t lo, hi;  // lowest / one past the highest typed byte of one instance
    int gran;        // power of two dividing every run, displacement and stride
    int64_t max_blen;  // longest run
};
// false: not a valid program
bool ddt_view_of(const ompi_amd_ddt_t *ddt, ddt_view *out);

}  // namespace ompi_amd
