// Device-side MPI_Op semantics shared by the op kernels and the fused
// collective reductions.  gfx950 only.
//
// f(x, y) is the reference's element rule with x = the OUT operand of the
// 2-buffer handler (inout) or in1 of the 3-buffer handler, y = in / in2:
//   ompi/mca/op/base/op_base_functions.c
//     OP_FUNC   :40-51   b = b op a            -> f(x,y) = x op y
//     FUNC_FUNC :60-73   b = current_func(b,a) -> MAX (x > y ? x : y) :153
//                                                 MIN (x < y ? x : y) :216
//     LOC_FUNC  :88-104, LOC_FUNC_3BUF :709-731 (differ; see loc2/loc3)
// MAX/MIN are compare+select, never v_max/v_min: NaN and ±0 must resolve to
// the second operand exactly as the C ternary does.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/ompi_amd.h"

namespace ompi_amd {

// MAXLOC/MINLOC pair types (op_base_functions.c:602-607); layouts match the
// C ABI (DOUBLE_INT: extent 16, v at 0, k at 8, 4 pad bytes).
struct float_int_t { float v; int k; };
struct double_int_t { double v; int k; };
struct long_int_t { long v; int k; };
struct two_int_t { int v; int k; };
struct short_int_t { short v; int k; };
static_assert(sizeof(double_int_t) == 16 && sizeof(short_int_t) == 8, "pair ABI");

// C complex types (MPI_C_FLOAT_COMPLEX / MPI_C_DOUBLE_COMPLEX): op/base
// reduces them with C99 `_Complex` arithmetic, OP_FUNC(sum|prod,
// c_float_complex, float _Complex, +=|*=) (op_base_functions.c:339-340,
// 408-409) and OP_FUNC_3BUF (:967-968, :1036-1037).  The product is GCC's
// C99 expansion: x = ac - bd, y = ad + bc in the element type, and only when
// both are NaN libgcc's __mul?c3 recovers the infinities (ISO C Annex G.5.1).
template <typename R> struct cplx {
    R re, im;
};
using cfloat_t = cplx<float>;
using cdouble_t = cplx<double>;
static_assert(sizeof(cfloat_t) == 8 && sizeof(cdouble_t) == 16, "complex ABI");

template <typename R>
__device__ __forceinline__ cplx<R> operator+(cplx<R> x, cplx<R> y) {
    return {x.re + y.re, x.im + y.im};
}

template <typename R> __device__ __forceinline__ R cp_inf_or_zero(R v) {
    return __builtin_copysign(__builtin_isinf(v) ? R(1) : R(0), v);
}
template <typename R> __device__ __forceinline__ R cp_nan_to_zero(R v) {
    return __builtin_isnan(v) ? __builtin_copysign(R(0), v) : v;
}

// (a + ib)(c + id); x = the first operand (2-buffer: out, 3-buffer: in1)
template <typename R>
__device__ __forceinline__ cplx<R> operator*(cplx<R> x, cplx<R> y) {
    R a = x.re, b = x.im, c = y.re, d = y.im;
    const R ac = a * c, bd = b * d, ad = a * d, bc = b * c;
    R re = ac - bd, im = ad + bc;
    if (__builtin_isnan(re) && __builtin_isnan(im)) {
        bool again = false;
        if (__builtin_isinf(a) || __builtin_isinf(b)) {
            a = cp_inf_or_zero(a);
            b = cp_inf_or_zero(b);
            c = cp_nan_to_zero(c);
            d = cp_nan_to_zero(d);
            again = true;
        }
        if (__builtin_isinf(c) || __builtin_isinf(d)) {
            c = cp_inf_or_zero(c);
            d = cp_inf_or_zero(d);
            a = cp_nan_to_zero(a);
            b = cp_nan_to_zero(b);
            again = true;
        }
        if (!again && (__builtin_isinf(ac) || __builtin_isinf(bd) || __builtin_isinf(ad) ||
                       __builtin_isinf(bc))) {
            a = cp_nan_to_zero(a);
            b = cp_nan_to_zero(b);
            c = cp_nan_to_zero(c);
            d = cp_nan_to_zero(d);
            again = true;
        }
        if (again) {
            const R inf = __builtin_huge_val();
            re = inf * (a * c - b * d);
            im = inf * (a * d + b * c);
        }
    }
    return {re, im};
}

// Short float (opal_short_float_t = _Float16, the MPIX_C_FLOAT16 extension)
// and its complex, opal_short_float_t[2]: op/base has no `short float
// _Complex`, so it reduces the pair with COMPLEX_SUM_FUNC / COMPLEX_PROD_FUNC
// (op_base_functions.c:112-147, 3-buffer :739-775):
//   sum   re = x.re + y.re, im = x.im + y.im
//   prod  re = y.re*x.re - y.im*x.im, im = y.re*x.im + y.im*x.re
// (y = in / in2 on the left as the reference writes it; every term below is
// commutative bit for bit).  On the x86-64 hosts MI355X nodes run, gcc and
// clang evaluate _Float16 expressions in float (excess precision, rounded
// once at the assignment): the products of two halves are exact in float
// (11 + 11 significant bits), the sum or difference rounds once to float,
// then to half.  The device does exactly that, so the result is the x86
// reference's bit for bit.  Real short float +, * and the compares are
// correctly rounded either way (float's 24 bits >= 2 x 11 + 2: rounding to
// float and then to half equals rounding to half once), so v_add_f16 /
// v_mul_f16 give the same bits as the host's float evaluation.
using half_t = _Float16;
struct chalf_t {
    half_t re, im;
};
static_assert(sizeof(chalf_t) == 4, "short float complex ABI");
__device__ __forceinline__ chalf_t operator+(chalf_t x, chalf_t y) {
    return {(half_t)(x.re + y.re), (half_t)(x.im + y.im)};
}
__device__ __forceinline__ chalf_t operator*(chalf_t x, chalf_t y) {
    const float a = (float)x.re, b = (float)x.im, c = (float)y.re, d = (float)y.im;
    // exact products: contraction into an fma cannot change the result
    return {(half_t)(c * a - d * b), (half_t)(c * b + d * a)};
}

template <typename T> struct is_pair { static constexpr bool value = false; };
template <> struct is_pair<float_int_t> { static constexpr bool value = true; };
template <> struct is_pair<double_int_t> { static constexpr bool value = true; };
template <> struct is_pair<long_int_t> { static constexpr bool value = true; };
template <> struct is_pair<two_int_t> { static constexpr bool value = true; };
template <> struct is_pair<short_int_t> { static constexpr bool value = true; };

// type code -> C type
template <int TYPE> struct type_of;
template <> struct type_of<OMPI_AMD_TYPE_INT8_T> { using type = int8_t; };
template <> struct type_of<OMPI_AMD_TYPE_UINT8_T> { using type = uint8_t; };
template <> struct type_of<OMPI_AMD_TYPE_INT16_T> { using type = int16_t; };
template <> struct type_of<OMPI_AMD_TYPE_UINT16_T> { using type = uint16_t; };
template <> struct type_of<OMPI_AMD_TYPE_INT32_T> { using type = int32_t; };
template <> struct type_of<OMPI_AMD_TYPE_UINT32_T> { using type = uint32_t; };
template <> struct type_of<OMPI_AMD_TYPE_INT64_T> { using type = int64_t; };
template <> struct type_of<OMPI_AMD_TYPE_UINT64_T> { using type = uint64_t; };
template <> struct type_of<OMPI_AMD_TYPE_SHORT_FLOAT> { using type = half_t; };
template <> struct type_of<OMPI_AMD_TYPE_FLOAT> { using type = float; };
template <> struct type_of<OMPI_AMD_TYPE_DOUBLE> { using type = double; };
template <> struct type_of<OMPI_AMD_TYPE_BOOL> { using type = bool; };
template <> struct type_of<OMPI_AMD_TYPE_BYTE> { using type = char; };
template <> struct type_of<OMPI_AMD_TYPE_FLOAT_INT> { using type = float_int_t; };
template <> struct type_of<OMPI_AMD_TYPE_DOUBLE_INT> { using type = double_int_t; };
template <> struct type_of<OMPI_AMD_TYPE_LONG_INT> { using type = long_int_t; };
template <> struct type_of<OMPI_AMD_TYPE_2INT> { using type = two_int_t; };
template <> struct type_of<OMPI_AMD_TYPE_SHORT_INT> { using type = short_int_t; };
template <> struct type_of<OMPI_AMD_TYPE_C_SHORT_FLOAT_COMPLEX> { using type = chalf_t; };
template <> struct type_of<OMPI_AMD_TYPE_C_FLOAT_COMPLEX> { using type = cfloat_t; };
template <> struct type_of<OMPI_AMD_TYPE_C_DOUBLE_COMPLEX> { using type = cdouble_t; };

// Which (op,type) slots exist — the op/base table pattern
// (op_base_functions.c:1485-1569) restricted to the predefined C types.
__host__ __device__ constexpr bool is_c_int(int t) { return t >= 0 && t <= 7; }
__host__ __device__ constexpr bool is_fp(int t) {
    return t == OMPI_AMD_TYPE_SHORT_FLOAT || t == OMPI_AMD_TYPE_FLOAT || t == OMPI_AMD_TYPE_DOUBLE;
}
__host__ __device__ constexpr bool is_pair_type(int t) {
    return t == OMPI_AMD_TYPE_FLOAT_INT || t == OMPI_AMD_TYPE_DOUBLE_INT ||
           t == OMPI_AMD_TYPE_LONG_INT || t == OMPI_AMD_TYPE_2INT || t == OMPI_AMD_TYPE_SHORT_INT;
}
__host__ __device__ constexpr bool is_c_complex(int t) {
    return t == OMPI_AMD_TYPE_C_SHORT_FLOAT_COMPLEX || t == OMPI_AMD_TYPE_C_FLOAT_COMPLEX ||
           t == OMPI_AMD_TYPE_C_DOUBLE_COMPLEX;
}
// (op/base's FLOATING_POINT and COMPLEX(sum|prod) rows,
// op_base_functions.c:1400-1406, 1432-1436, as filled when configure finds
// _Float16; long double and its complex stay with op/base: gfx950 has no
// long double)
__host__ __device__ constexpr bool slot_supported(int op, int t) {
    return (op == OMPI_AMD_OP_SUM || op == OMPI_AMD_OP_PROD) && is_c_complex(t) ? true
         : (op == OMPI_AMD_OP_MAX || op == OMPI_AMD_OP_MIN || op == OMPI_AMD_OP_SUM ||
            op == OMPI_AMD_OP_PROD) ? (is_c_int(t) || is_fp(t))
         : (op == OMPI_AMD_OP_LAND || op == OMPI_AMD_OP_LOR || op == OMPI_AMD_OP_LXOR)
               ? (is_c_int(t) || t == OMPI_AMD_TYPE_BOOL)
         : (op == OMPI_AMD_OP_BAND || op == OMPI_AMD_OP_BOR || op == OMPI_AMD_OP_BXOR)
               ? (is_c_int(t) || t == OMPI_AMD_TYPE_BYTE)
         : (op == OMPI_AMD_OP_MAXLOC || op == OMPI_AMD_OP_MINLOC) ? is_pair_type(t)
                                                                 : false;
}

// Element rule.  THREE selects the 3-buffer LOC variant (it returns in2 on
// an unordered compare; the 2-buffer one keeps out).
template <int OP, bool THREE> struct opfn;

#define OMPI_AMD_ARITH(OPC, EXPR)                                              \
    template <bool THREE> struct opfn<OPC, THREE> {                           \
        template <typename T> __device__ __forceinline__ static T f(T x, T y) { return (T)(EXPR); } \
    };
OMPI_AMD_ARITH(OMPI_AMD_OP_SUM, x + y)
OMPI_AMD_ARITH(OMPI_AMD_OP_PROD, x * y)
OMPI_AMD_ARITH(OMPI_AMD_OP_MAX, (x > y) ? x : y)
OMPI_AMD_ARITH(OMPI_AMD_OP_MIN, (x < y) ? x : y)
OMPI_AMD_ARITH(OMPI_AMD_OP_LAND, x && y)
OMPI_AMD_ARITH(OMPI_AMD_OP_LOR, x || y)
OMPI_AMD_ARITH(OMPI_AMD_OP_LXOR, (x ? 1 : 0) ^ (y ? 1 : 0))
OMPI_AMD_ARITH(OMPI_AMD_OP_BAND, x & y)
OMPI_AMD_ARITH(OMPI_AMD_OP_BOR, x | y)
OMPI_AMD_ARITH(OMPI_AMD_OP_BXOR, x ^ y)
#undef OMPI_AMD_ARITH

template <int OP, bool THREE> struct locfn {
    template <typename S> __device__ __forceinline__ static S f(S x, S y) {
        S r = x;  // keeps x's gap bytes (2-buffer: x = out)
        if (!THREE) {
            // LOC_FUNC: a = in = y, b = out = x
            const bool take = (OP == OMPI_AMD_OP_MAXLOC) ? (y.v > x.v) : (y.v < x.v);
            if (take) { r.v = y.v; r.k = y.k; }
            else if (y.v == x.v) { r.k = (x.k < y.k) ? x.k : y.k; }
        } else {
            // LOC_FUNC_3BUF: a1 = x, a2 = y
            const bool take = (OP == OMPI_AMD_OP_MAXLOC) ? (x.v > y.v) : (x.v < y.v);
            if (take) { /* r = x */ }
            else if (x.v == y.v) { r.k = (y.k < x.k) ? y.k : x.k; }
            else { r.v = y.v; r.k = y.k; }
        }
        return r;
    }
};
template <bool THREE> struct opfn<OMPI_AMD_OP_MAXLOC, THREE> : locfn<OMPI_AMD_OP_MAXLOC, THREE> {};
template <bool THREE> struct opfn<OMPI_AMD_OP_MINLOC, THREE> : locfn<OMPI_AMD_OP_MINLOC, THREE> {};

// 16-byte vector used for every global access on the streaming paths.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <typename T> union vec16 {
    u32x4 v;
    T e[16 / sizeof(T)];
};

// Store one element.  For the gapped pair types (DOUBLE_INT, LONG_INT,
// SHORT_INT) the gap bytes carry whatever the first operand held: padding
// takes unspecified values whenever a member is stored (C11 6.2.6.1p6), so
// op/base itself gives no guarantee on them either.
template <typename T>
__device__ __forceinline__ void store_elem(T *p, const T &r) {
    *p = r;
}

}  // namespace ompi_amd
