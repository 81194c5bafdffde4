/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Scalar restatement of op/base's 2-buffer and 3-buffer reduction handlers
 * for the predefined C types.  Semantics, per element:
 *
 *   2-buffer (ompi/mca/op/base/op_base_functions.c)
 *     SUM/PROD          b = b + a / b = b * a            OP_FUNC      :40-51
 *     MAX/MIN           b = (b > a) ? b : a  (b<a for MIN) FUNC_FUNC  :60-73,153-154,216
 *     LAND/LOR/LXOR     b && a, b || a, (b?1:0)^(a?1:0)  FUNC_FUNC    :416-470
 *     BAND/BOR/BXOR     b & a, b | a, b ^ a              FUNC_FUNC    :482-587
 *     MAXLOC/MINLOC     if (a.v > b.v) b = a; else if (a.v == b.v)
 *                       b.k = min(b.k, a.k)              LOC_FUNC     :88-104
 *   where a = in[i], b = inout[i].
 *
 *   3-buffer (same file)
 *     OP/FUNC           out = in1 (op) in2               :654-692
 *     LOC               if (a1.v op a2.v) out = a1; else if equal
 *                       out = {a1.v, min(a2.k, a1.k)}; else out = a2  :709-731
 *
 *   C complex (float / double _Complex, :339-340, :408-409, :967-968,
 *   :1036-1037): SUM and PROD only, with C99 `_Complex` arithmetic exactly
 *   as op/base writes it (`*b *= *a`, `out = in1 * in2`); gcc's expansion
 *   of the product (x = ac - bd, y = ad + bc, libgcc's __mul?c3 recovery
 *   when both are NaN, ISO C Annex G.5.1) is what the reference computes.
 *
 *   Short float (opal_short_float_t = _Float16 wherever configure finds
 *   it, config/opal_check_alt_short_float.m4:27-35): SUM/PROD/MAX/MIN
 *   (:184-187, :247-250, :307-310, :376-379, 3-buffer :813-815, :876-878,
 *   :936-938, :1005-1007) and its complex, opal_short_float_t[2], SUM/PROD
 *   through COMPLEX_SUM_FUNC / COMPLEX_PROD_FUNC (:112-147, :334-337,
 *   :403-406, 3-buffer :739-775, :963-965, :1032-1034):
 *     re = a.re*b.re - a.im*b.im, im = a.re*b.im + a.im*b.re  (a = in)
 *   An x86-64 gcc/clang build evaluates _Float16 expressions in float and
 *   rounds once at the assignment (no native half arithmetic below
 *   AVX512-FP16); restated here with explicit float arithmetic and
 *   orc_f2h.  For a single +, * that equals rounding to half directly
 *   (24 >= 2*11 + 2 bits), for the complex product it is the x86 result.
 *
 * Note the NaN / signed-zero consequences (pinned in tests/golden):
 * MAX(out=x, in=NaN) = NaN, MAX(out=NaN, in=3) = 3, MAX(out=+0,in=-0) = -0.
 * LOC handlers only write v and k, never the struct padding.
 */
#include "oracle.h"

#include <complex.h>
#include <string.h>
#include <time.h>

typedef struct { float v; int k; } orc_float_int_t;     /* size 8  */
typedef struct { double v; int k; } orc_double_int_t;   /* extent 16, 12 used */
typedef struct { long v; int k; } orc_long_int_t;       /* extent 16, 12 used */
typedef struct { int v; int k; } orc_2int_t;            /* size 8  */
typedef struct { short v; int k; } orc_short_int_t;     /* extent 8, 6 used */

size_t orc_type_extent(int type)
{
    switch (type) {
    case ORC_T_INT8: case ORC_T_UINT8: case ORC_T_BOOL: case ORC_T_BYTE: return 1;
    case ORC_T_INT16: case ORC_T_UINT16: case ORC_T_SHORT_FLOAT: return 2;
    case ORC_T_INT32: case ORC_T_UINT32: case ORC_T_FLOAT: case ORC_T_C_SHORT_FLOAT_COMPLEX: return 4;
    case ORC_T_INT64: case ORC_T_UINT64: case ORC_T_DOUBLE: return 8;
    case ORC_T_FLOAT_INT: return sizeof(orc_float_int_t);
    case ORC_T_DOUBLE_INT: return sizeof(orc_double_int_t);
    case ORC_T_LONG_INT: return sizeof(orc_long_int_t);
    case ORC_T_2INT: return sizeof(orc_2int_t);
    case ORC_T_SHORT_INT: return sizeof(orc_short_int_t);
    case ORC_T_C_FLOAT_COMPLEX: return sizeof(float _Complex);
    case ORC_T_C_DOUBLE_COMPLEX: return sizeof(double _Complex);
    default: return 0;
    }
}

static int is_c_int(int t) { return t >= ORC_T_INT8 && t <= ORC_T_UINT64; }
static int is_fp(int t) { return t == ORC_T_SHORT_FLOAT || t == ORC_T_FLOAT || t == ORC_T_DOUBLE; }
static int is_complex(int t)
{
    return t == ORC_T_C_SHORT_FLOAT_COMPLEX || t == ORC_T_C_FLOAT_COMPLEX || t == ORC_T_C_DOUBLE_COMPLEX;
}

/* ---- binary16 ---- */
float orc_h2f(uint16_t h)
{
    uint32_t s = (uint32_t)(h & 0x8000u) << 16, e = (h >> 10) & 0x1fu, m = h & 0x3ffu, x;
    float f;
    if (e == 0) {
        if (m == 0) {
            x = s;
        } else { /* subnormal half: normalise into a float */
            uint32_t sh = 0;
            while (!(m & 0x400u)) { m <<= 1; sh++; }
            x = s | ((113u - sh) << 23) | ((m & 0x3ffu) << 13);
        }
    } else if (e == 31) {
        x = s | 0x7f800000u | (m << 13);
    } else {
        x = s | ((e + 112u) << 23) | (m << 13);
    }
    memcpy(&f, &x, 4);
    return f;
}

uint16_t orc_f2h(float f)
{
    uint32_t x, ax, sign, e, m, q, rem, half;
    int shift;
    memcpy(&x, &f, 4);
    sign = (x >> 16) & 0x8000u;
    ax = x & 0x7fffffffu;
    if (ax >= 0x7f800000u) /* inf; NaN stays NaN (quiet, top payload bits) */
        return (uint16_t)(sign | (ax == 0x7f800000u ? 0x7c00u : 0x7e00u | ((ax >> 13) & 0x3ffu)));
    if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u); /* >= 65520: inf */
    if (ax >= 0x38800000u) { /* normal half: drop 13 bits, nearest even */
        q = (ax - 0x38000000u) >> 13;
        rem = ax & 0x1fffu;
        q += (rem > 0x1000u || (rem == 0x1000u && (q & 1u))) ? 1u : 0u;
        return (uint16_t)(sign | q);
    }
    e = ax >> 23;
    if (e == 0) return (uint16_t)sign; /* float subnormal: far below 2^-25 */
    m = (ax & 0x7fffffu) | 0x800000u;  /* value = m * 2^(e-150) = (m * 2^(e-126)) * 2^-24 */
    shift = 126 - (int)e;
    if (shift > 24) return (uint16_t)sign;
    q = m >> shift;
    rem = m & ((1u << shift) - 1u);
    half = 1u << (shift - 1);
    q += (rem > half || (rem == half && (q & 1u))) ? 1u : 0u;
    return (uint16_t)(sign | q);
}
static int is_loc(int t)
{
    return t == ORC_T_FLOAT_INT || t == ORC_T_DOUBLE_INT || t == ORC_T_LONG_INT ||
           t == ORC_T_2INT || t == ORC_T_SHORT_INT;
}

/* Which slots op/base fills (op_base_functions.c:1485-1569). */
int orc_op_defined(int op, int type)
{
    switch (op) {
    case ORC_OP_SUM: case ORC_OP_PROD:
        return is_c_int(type) || is_fp(type) || is_complex(type);
    case ORC_OP_MAX: case ORC_OP_MIN:
        return is_c_int(type) || is_fp(type);
    case ORC_OP_LAND: case ORC_OP_LOR: case ORC_OP_LXOR:
        return is_c_int(type) || type == ORC_T_BOOL;
    case ORC_OP_BAND: case ORC_OP_BOR: case ORC_OP_BXOR:
        return is_c_int(type) || type == ORC_T_BYTE;
    case ORC_OP_MAXLOC: case ORC_OP_MINLOC:
        return is_loc(type);
    default:
        return 0;
    }
}

/* ---- element loops; b = out (2buff) / x = in1 (3buff) ---- */
#define ORC_ARITH_LOOPS(T)                                                     \
    static void arith2_##T(int op, const T *a, T *b, size_t n)                 \
    {                                                                          \
        size_t i;                                                              \
        switch (op) {                                                          \
        case ORC_OP_SUM: for (i = 0; i < n; i++) b[i] = (T)(b[i] + a[i]); break; \
        case ORC_OP_PROD: for (i = 0; i < n; i++) b[i] = (T)(b[i] * a[i]); break; \
        case ORC_OP_MAX: for (i = 0; i < n; i++) b[i] = (b[i] > a[i]) ? b[i] : a[i]; break; \
        case ORC_OP_MIN: for (i = 0; i < n; i++) b[i] = (b[i] < a[i]) ? b[i] : a[i]; break; \
        }                                                                      \
    }                                                                          \
    static void arith3_##T(int op, const T *x, const T *y, T *o, size_t n)     \
    {                                                                          \
        size_t i;                                                              \
        switch (op) {                                                          \
        case ORC_OP_SUM: for (i = 0; i < n; i++) o[i] = (T)(x[i] + y[i]); break; \
        case ORC_OP_PROD: for (i = 0; i < n; i++) o[i] = (T)(x[i] * y[i]); break; \
        case ORC_OP_MAX: for (i = 0; i < n; i++) o[i] = (x[i] > y[i]) ? x[i] : y[i]; break; \
        case ORC_OP_MIN: for (i = 0; i < n; i++) o[i] = (x[i] < y[i]) ? x[i] : y[i]; break; \
        }                                                                      \
    }

#define ORC_BIT_LOOPS(T)                                                       \
    static void bits2_##T(int op, const T *a, T *b, size_t n)                  \
    {                                                                          \
        size_t i;                                                              \
        switch (op) {                                                          \
        case ORC_OP_LAND: for (i = 0; i < n; i++) b[i] = (T)(b[i] && a[i]); break; \
        case ORC_OP_LOR: for (i = 0; i < n; i++) b[i] = (T)(b[i] || a[i]); break; \
        case ORC_OP_LXOR: for (i = 0; i < n; i++) b[i] = (T)((b[i] ? 1 : 0) ^ (a[i] ? 1 : 0)); break; \
        case ORC_OP_BAND: for (i = 0; i < n; i++) b[i] = (T)(b[i] & a[i]); break; \
        case ORC_OP_BOR: for (i = 0; i < n; i++) b[i] = (T)(b[i] | a[i]); break; \
        case ORC_OP_BXOR: for (i = 0; i < n; i++) b[i] = (T)(b[i] ^ a[i]); break; \
        }                                                                      \
    }                                                                          \
    static void bits3_##T(int op, const T *x, const T *y, T *o, size_t n)      \
    {                                                                          \
        size_t i;                                                              \
        switch (op) {                                                          \
        case ORC_OP_LAND: for (i = 0; i < n; i++) o[i] = (T)(x[i] && y[i]); break; \
        case ORC_OP_LOR: for (i = 0; i < n; i++) o[i] = (T)(x[i] || y[i]); break; \
        case ORC_OP_LXOR: for (i = 0; i < n; i++) o[i] = (T)((x[i] ? 1 : 0) ^ (y[i] ? 1 : 0)); break; \
        case ORC_OP_BAND: for (i = 0; i < n; i++) o[i] = (T)(x[i] & y[i]); break; \
        case ORC_OP_BOR: for (i = 0; i < n; i++) o[i] = (T)(x[i] | y[i]); break; \
        case ORC_OP_BXOR: for (i = 0; i < n; i++) o[i] = (T)(x[i] ^ y[i]); break; \
        }                                                                      \
    }

#define ORC_LOC_LOOPS(S)                                                       \
    static void loc2_##S(int op, const S *a, S *b, size_t n)                   \
    {                                                                          \
        size_t i;                                                              \
        for (i = 0; i < n; i++) {                                              \
            int take = (op == ORC_OP_MAXLOC) ? (a[i].v > b[i].v) : (a[i].v < b[i].v); \
            if (take) {                                                        \
                b[i].v = a[i].v;                                               \
                b[i].k = a[i].k;                                               \
            } else if (a[i].v == b[i].v) {                                     \
                b[i].k = (b[i].k < a[i].k) ? b[i].k : a[i].k;                  \
            }                                                                  \
        }                                                                      \
    }                                                                          \
    static void loc3_##S(int op, const S *x, const S *y, S *o, size_t n)       \
    {                                                                          \
        size_t i;                                                              \
        for (i = 0; i < n; i++) {                                              \
            int take = (op == ORC_OP_MAXLOC) ? (x[i].v > y[i].v) : (x[i].v < y[i].v); \
            if (take) {                                                        \
                o[i].v = x[i].v;                                               \
                o[i].k = x[i].k;                                               \
            } else if (x[i].v == y[i].v) {                                     \
                o[i].v = x[i].v;                                               \
                o[i].k = (y[i].k < x[i].k) ? y[i].k : x[i].k;                  \
            } else {                                                           \
                o[i].v = y[i].v;                                               \
                o[i].k = y[i].k;                                               \
            }                                                                  \
        }                                                                      \
    }

ORC_ARITH_LOOPS(int8_t) ORC_ARITH_LOOPS(uint8_t) ORC_ARITH_LOOPS(int16_t)
ORC_ARITH_LOOPS(uint16_t) ORC_ARITH_LOOPS(int32_t) ORC_ARITH_LOOPS(uint32_t)
ORC_ARITH_LOOPS(int64_t) ORC_ARITH_LOOPS(uint64_t)
typedef float orc_f32; typedef double orc_f64;
ORC_ARITH_LOOPS(orc_f32) ORC_ARITH_LOOPS(orc_f64)

ORC_BIT_LOOPS(int8_t) ORC_BIT_LOOPS(uint8_t) ORC_BIT_LOOPS(int16_t)
ORC_BIT_LOOPS(uint16_t) ORC_BIT_LOOPS(int32_t) ORC_BIT_LOOPS(uint32_t)
ORC_BIT_LOOPS(int64_t) ORC_BIT_LOOPS(uint64_t)
typedef _Bool orc_bool; typedef char orc_byte;
ORC_BIT_LOOPS(orc_bool) ORC_BIT_LOOPS(orc_byte)

/* short float: float evaluation, one rounding (see the header comment) */
static uint16_t h_arith(int op, uint16_t x, uint16_t y) /* x = out / in1, y = in / in2 */
{
    const float fx = orc_h2f(x), fy = orc_h2f(y);
    switch (op) {
    case ORC_OP_SUM: return orc_f2h(fx + fy);
    case ORC_OP_PROD: return orc_f2h(fx * fy);
    case ORC_OP_MAX: return (fx > fy) ? x : y;
    default: return (fx < fy) ? x : y; /* MIN */
    }
}
static void arith2_half(int op, const uint16_t *a, uint16_t *b, size_t n)
{
    size_t i;
    for (i = 0; i < n; i++) b[i] = h_arith(op, b[i], a[i]);
}
static void arith3_half(int op, const uint16_t *x, const uint16_t *y, uint16_t *o, size_t n)
{
    size_t i;
    for (i = 0; i < n; i++) o[i] = h_arith(op, x[i], y[i]);
}
/* opal_short_float_t[2]: COMPLEX_SUM_FUNC / COMPLEX_PROD_FUNC; a = in (2buff)
 * or in1 (3buff), b = out (2buff) or in2 (3buff), written as the reference
 * writes them */
static void chalf(int op, const uint16_t *a, const uint16_t *b, uint16_t *o)
{
    const float a0 = orc_h2f(a[0]), a1 = orc_h2f(a[1]), b0 = orc_h2f(b[0]), b1 = orc_h2f(b[1]);
    uint16_t r0, r1;
    if (op == ORC_OP_SUM) {
        r0 = orc_f2h(b0 + a0);
        r1 = orc_f2h(b1 + a1);
    } else {
        r0 = orc_f2h(a0 * b0 - a1 * b1);
        r1 = orc_f2h(a0 * b1 + a1 * b0);
    }
    o[0] = r0;
    o[1] = r1;
}
static void cplx2_c16(int op, const uint16_t *a, uint16_t *b, size_t n)
{
    size_t i;
    for (i = 0; i < n; i++) chalf(op, a + 2 * i, b + 2 * i, b + 2 * i);
}
static void cplx3_c16(int op, const uint16_t *x, const uint16_t *y, uint16_t *o, size_t n)
{
    size_t i;
    for (i = 0; i < n; i++) chalf(op, x + 2 * i, y + 2 * i, o + 2 * i);
}

/* OP_FUNC / OP_FUNC_3BUF over the C complex types: SUM and PROD only */
#define ORC_COMPLEX_LOOPS(NAME, T)                                             \
    static void cplx2_##NAME(int op, const T *a, T *b, size_t n)               \
    {                                                                          \
        size_t i;                                                              \
        if (op == ORC_OP_SUM) for (i = 0; i < n; i++) b[i] += a[i];            \
        else for (i = 0; i < n; i++) b[i] *= a[i];                             \
    }                                                                          \
    static void cplx3_##NAME(int op, const T *x, const T *y, T *o, size_t n)   \
    {                                                                          \
        size_t i;                                                              \
        if (op == ORC_OP_SUM) for (i = 0; i < n; i++) o[i] = x[i] + y[i];      \
        else for (i = 0; i < n; i++) o[i] = x[i] * y[i];                       \
    }
ORC_COMPLEX_LOOPS(c32, float _Complex)
ORC_COMPLEX_LOOPS(c64, double _Complex)

ORC_LOC_LOOPS(orc_float_int_t) ORC_LOC_LOOPS(orc_double_int_t)
ORC_LOC_LOOPS(orc_long_int_t) ORC_LOC_LOOPS(orc_2int_t)
ORC_LOC_LOOPS(orc_short_int_t)

static int is_arith(int op)
{
    return op == ORC_OP_SUM || op == ORC_OP_PROD || op == ORC_OP_MAX || op == ORC_OP_MIN;
}

#define DISPATCH_INT(FAM, ARGS2, ...)                                          \
    switch (type) {                                                            \
    case ORC_T_INT8: FAM##_int8_t ARGS2; return 0;                             \
    case ORC_T_UINT8: FAM##_uint8_t ARGS2; return 0;                           \
    case ORC_T_INT16: FAM##_int16_t ARGS2; return 0;                           \
    case ORC_T_UINT16: FAM##_uint16_t ARGS2; return 0;                         \
    case ORC_T_INT32: FAM##_int32_t ARGS2; return 0;                           \
    case ORC_T_UINT32: FAM##_uint32_t ARGS2; return 0;                         \
    case ORC_T_INT64: FAM##_int64_t ARGS2; return 0;                           \
    case ORC_T_UINT64: FAM##_uint64_t ARGS2; return 0;                         \
    __VA_ARGS__                                                                \
    default: return -1;                                                        \
    }

int orc_op_2buff(int op, int type, const void *in, void *inout, size_t count)
{
    if (!orc_op_defined(op, type)) return -1;
    if (op == ORC_OP_MAXLOC || op == ORC_OP_MINLOC) {
        switch (type) {
        case ORC_T_FLOAT_INT: loc2_orc_float_int_t(op, in, inout, count); return 0;
        case ORC_T_DOUBLE_INT: loc2_orc_double_int_t(op, in, inout, count); return 0;
        case ORC_T_LONG_INT: loc2_orc_long_int_t(op, in, inout, count); return 0;
        case ORC_T_2INT: loc2_orc_2int_t(op, in, inout, count); return 0;
        case ORC_T_SHORT_INT: loc2_orc_short_int_t(op, in, inout, count); return 0;
        default: return -1;
        }
    }
    if (type == ORC_T_C_SHORT_FLOAT_COMPLEX) { cplx2_c16(op, in, inout, count); return 0; }
    if (type == ORC_T_SHORT_FLOAT) { arith2_half(op, in, inout, count); return 0; }
    if (type == ORC_T_C_FLOAT_COMPLEX) { cplx2_c32(op, in, inout, count); return 0; }
    if (type == ORC_T_C_DOUBLE_COMPLEX) { cplx2_c64(op, in, inout, count); return 0; }
    if (is_arith(op)) {
        DISPATCH_INT(arith2, (op, in, inout, count),
                     case ORC_T_FLOAT: arith2_orc_f32(op, in, inout, count); return 0;
                     case ORC_T_DOUBLE: arith2_orc_f64(op, in, inout, count); return 0;)
    }
    DISPATCH_INT(bits2, (op, in, inout, count),
                 case ORC_T_BOOL: bits2_orc_bool(op, in, inout, count); return 0;
                 case ORC_T_BYTE: bits2_orc_byte(op, in, inout, count); return 0;)
}

int orc_op_3buff(int op, int type, const void *in1, const void *in2, void *out,
                 size_t count)
{
    if (!orc_op_defined(op, type)) return -1;
    if (op == ORC_OP_MAXLOC || op == ORC_OP_MINLOC) {
        switch (type) {
        case ORC_T_FLOAT_INT: loc3_orc_float_int_t(op, in1, in2, out, count); return 0;
        case ORC_T_DOUBLE_INT: loc3_orc_double_int_t(op, in1, in2, out, count); return 0;
        case ORC_T_LONG_INT: loc3_orc_long_int_t(op, in1, in2, out, count); return 0;
        case ORC_T_2INT: loc3_orc_2int_t(op, in1, in2, out, count); return 0;
        case ORC_T_SHORT_INT: loc3_orc_short_int_t(op, in1, in2, out, count); return 0;
        default: return -1;
        }
    }
    if (type == ORC_T_C_SHORT_FLOAT_COMPLEX) { cplx3_c16(op, in1, in2, out, count); return 0; }
    if (type == ORC_T_SHORT_FLOAT) { arith3_half(op, in1, in2, out, count); return 0; }
    if (type == ORC_T_C_FLOAT_COMPLEX) { cplx3_c32(op, in1, in2, out, count); return 0; }
    if (type == ORC_T_C_DOUBLE_COMPLEX) { cplx3_c64(op, in1, in2, out, count); return 0; }
    if (is_arith(op)) {
        DISPATCH_INT(arith3, (op, in1, in2, out, count),
                     case ORC_T_FLOAT: arith3_orc_f32(op, in1, in2, out, count); return 0;
                     case ORC_T_DOUBLE: arith3_orc_f64(op, in1, in2, out, count); return 0;)
    }
    DISPATCH_INT(bits3, (op, in1, in2, out, count),
                 case ORC_T_BOOL: bits3_orc_bool(op, in1, in2, out, count); return 0;
                 case ORC_T_BYTE: bits3_orc_byte(op, in1, in2, out, count); return 0;)
}

double orc_time_op_3buff(int op, int type, const void *in1, const void *in2,
                         void *out, size_t count, int iters)
{
    struct timespec t0, t1;
    int it;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (it = 0; it < iters; it++) orc_op_3buff(op, type, in1, in2, out, count);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
