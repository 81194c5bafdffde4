"""Generate the committed golden fixtures in tests/golden/.

Sources (all restated, nothing executed from /root/reference):

* op_kat.json — the known-answer tests of test/datatype/reduce_local.c:
  constant inputs per type family (:195-199, :329-330, :459-460, :589-590,
  :739-740, :869-870, :999-1000, :1129-1130, :1262-1263, :1338-1339), the
  C expression each op is checked with (:209-217 and siblings; MIN is
  called with in/out swapped on purpose, :239-240), and the element counts
  of test/datatype/check_op.sh:27-30 (1 MiB + {0,1,7,15,31,63,127,130}) and
  of reduce_local's default sweep (1..1e6 doubling, :82).
* op_edge.json — outputs of the reference's compiled op_base_functions.c
  recorded in SURVEY.md §8(c) (NaN / ±0 / MAXLOC tie behaviour).
* ring_closed_form.json — the allreduce summation orders the survey
  verified against coll_base_allreduce.c (§8(c)): ring block b =
  x[b-1] + (x[b-2] + (... + (x[b+1] + x[b]))); recursive doubling (pof2) =
  pairwise tree.  Evaluated here in numpy float32, independently of the C
  oracle, on inputs chosen so the two orders round differently.
* unpack_ooo.json — test/datatype/unpack_ooo.c: the struct of strided int
  and double vectors (:167-266) over struct foo_t (:30-33), the packed
  input pbar and the receive buffer bar as the test initialises them
  (:80-92), the expected result it checks (:125-131), and its four
  fragment tables of (bytes, offset) pairs (:199-250), as data.
* ddt_kat.json — the datatypes of test/datatype/ddt_lib.c / ddt_test.c
  (vector(450,10,11) of double :479-493; blacs indexed :273-300; upper
  triangular(100) :130-144; struct{char,double} :230-245; vector(2,2,5)
  :248-257) as flattened typemaps with their MPI size/extent and the
  chunk sizes those tests drive the convertor with.

Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import struct

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

# OMPI_OP_BASE_FORTRAN_*
MAX, MIN, SUM, PROD, BAND, BOR, BXOR = 1, 2, 3, 4, 6, 8, 10
OPNAME = {MAX: "max", MIN: "min", SUM: "sum", PROD: "prod", BAND: "band", BOR: "bor",
          BXOR: "bxor"}

# (type code, numpy dtype, in, inout, reduce_local.c lines)
FAMILIES = [
    (0, "int8", 5, -3, "reduce_local.c:193-199"),
    (2, "int16", 5, -3, "reduce_local.c:324-330"),
    (4, "int32", 5, 3, "reduce_local.c:454-460"),
    (6, "int64", 5, 3, "reduce_local.c:584-590"),
    (1, "uint8", 5, 121, "reduce_local.c:734-740"),
    (3, "uint16", 5, 1234, "reduce_local.c:864-870"),
    (5, "uint32", 5, 3, "reduce_local.c:994-1000"),
    (7, "uint64", 5, 32433, "reduce_local.c:1124-1130"),
    (15, "float32", 1000.0 + 1, 100.0 + 2, "reduce_local.c:1257-1263"),
    (16, "float64", 10.0 + 1, 1.0 + 2, "reduce_local.c:1333-1339"),
]

INT_OPS = [MAX, MIN, SUM, PROD, BAND, BOR, BXOR]  # check_op.sh:19
FP_OPS = [MAX, MIN, SUM, PROD]                    # check_op.sh:61,73
INT_COUNTS = [1024 * 1024 + s for s in (0, 1, 7, 15, 31, 63, 127, 130)]  # check_op.sh:27-30
FP_COUNTS = [1024 * 1024 + s for s in (1024, 127, 130)]                 # check_op.sh:63,75
SWEEP_COUNTS = [1 << k for k in range(20)]                               # reduce_local.c:82, 189


def kat_expected(op, dt, a_in, a_inout):
    """The C check expression of reduce_local.c for (op), in numpy `dt`."""
    t = np.dtype(dt).type
    i, o = t(a_in), t(a_inout)
    with np.errstate(over="ignore"):
        if op == SUM:
            return t(o + i)
        if op == PROD:
            return t(i * o)
        if op == MAX:
            return o if o > i else i
        if op == MIN:
            return o if o < i else i
        if op == BAND:
            return t(i & o)
        if op == BOR:
            return t(i | o)
        if op == BXOR:
            return t(i ^ o)
    raise ValueError(op)


def op_kat():
    cases = []
    for code, dt, a_in, a_inout, ref in FAMILIES:
        fp = dt.startswith("float")
        for op in (FP_OPS if fp else INT_OPS):
            exp = kat_expected(op, dt, a_in, a_inout)
            if op == MIN:
                # MPI_Reduce_local(inout_buf, in_buf, ...): source holds the
                # inout constant, the target the in constant (:239-240)
                source, target = a_inout, a_in
            else:
                source, target = a_in, a_inout
            cases.append({
                "type_code": code, "dtype": dt, "op": op, "op_name": OPNAME[op],
                "source": source, "target": target,
                "expected_target": exp.item() if hasattr(exp, "item") else exp,
                "counts": (FP_COUNTS if fp else INT_COUNTS),
                "ref": ref + " + check_op.sh",
            })
    return {"sweep_counts": SWEEP_COUNTS, "cases": cases}


def f32bits(x):
    return struct.unpack("<I", struct.pack("<f", x))[0]


def op_edge():
    nan = float("nan")
    return {
        "ref": "SURVEY.md §8(c): compiled ompi/mca/op/base/op_base_functions.c, "
               "ompi_op_base_functions[MAX][FLOAT](in,out,&n,...)",
        "max_float_2buff": [
            # out, in -> out'
            {"out": f32bits(2.0), "in": f32bits(1.0), "result": f32bits(2.0)},
            {"out": f32bits(1.0), "in": f32bits(nan), "result": f32bits(nan)},
            {"out": f32bits(0.0), "in": f32bits(-0.0), "result": f32bits(-0.0)},
            {"out": f32bits(nan), "in": f32bits(3.0), "result": f32bits(3.0)},
        ],
        "maxloc_double_int_2buff": [
            {"out": [1.0, 5], "in": [1.0, 3], "result": [1.0, 3]},
        ],
        "double_int_sizeof": 16,
    }


def ring_closed_form():
    """Inputs where fp32 association order changes the bits."""
    rng = np.random.default_rng(20261015)
    out = {"ref": "SURVEY.md §8(c) ring / recursive-doubling closed forms", "cases": []}
    for n in (2, 4, 8):
        count = 3 * n + (n // 2)  # ragged: first count%n blocks one longer
        x = (rng.standard_normal((n, count)) * np.float32(1e3)).astype(np.float32)
        x[:, ::3] *= np.float32(1e-4)
        # block partition COLL_BASE_COMPUTE_BLOCKCOUNT
        early = late = count // n
        split = count % n
        if split:
            early += 1

        def boff(b):
            return b * early if b < split else b * late + split

        def bcnt(b):
            return early if b < split else late

        ring = np.empty(count, dtype=np.float32)
        for b in range(n):
            sl = slice(boff(b), boff(b) + bcnt(b))
            acc = x[b, sl].copy()
            for j in range(1, n):
                acc = (x[(b + j) % n, sl] + acc).astype(np.float32)
            ring[sl] = acc
        # pairwise tree (pof2)
        level = [x[r].copy() for r in range(n)]
        while len(level) > 1:
            level = [(level[2 * i + 1] + level[2 * i]).astype(np.float32)
                     for i in range(len(level) // 2)]
        tree = level[0]
        out["cases"].append({
            "nranks": n, "count": count,
            "x_bits": x.view(np.uint32).tolist(),
            "ring_bits": ring.view(np.uint32).tolist(),
            "tree_bits": tree.view(np.uint32).tolist(),
            "orders_differ": bool((ring.view(np.uint32) != tree.view(np.uint32)).any()),
        })
    return out


def ddt_kat():
    dbl = 8
    types = []
    # vector(450, 10, 11) of MPI_DOUBLE (ddt_test.c:479-493)
    types.append({
        "name": "vector_450_10_11_double", "ref": "ddt_test.c:479-493, ddt_lib.c create_vector_type",
        "blocks": [[i * 11 * dbl, 10 * dbl] for i in range(450)],
        "extent": (449 * 11 + 10) * dbl, "size": 450 * 10 * dbl, "count": 1,
        "chunks": [12, 82, 6000, 36000],
    })
    # blacs indexed of MPI_INT (ddt_lib.c:273-300)
    lens = [13, 13, 13, 13, 13, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1]
    disps = [1144, 1232, 1320, 1408, 1496, 1584, 1676, 1768, 1860, 1952, 2044, 2136, 2228,
             2320, 2412, 2504, 2596, 2688]
    types.append({
        "name": "blacs_indexed_int", "ref": "ddt_lib.c:273-300, ddt_test.c:516-528",
        "blocks": [[d, l * 4] for d, l in zip(disps, lens)],
        "extent": (2688 + 4) - 1144, "size": sum(lens) * 4, "count": 4500,
        "chunks": [956, 16 * 1024, 64 * 1024],
    })
    # upper triangular 100x100 double (ddt_lib.c:123-144)
    n = 100
    types.append({
        "name": "upper_matrix_100", "ref": "ddt_lib.c:123-144, opal_datatype_test.c",
        "blocks": [[(i * n + i) * dbl, (n - i) * dbl] for i in range(n)],
        "extent": n * n * dbl, "size": n * (n + 1) // 2 * dbl, "count": 1,
        "chunks": [48, 956],
    })
    # struct { char c; double d; } (ddt_lib.c:230-245)
    types.append({
        "name": "struct_char_double", "ref": "ddt_lib.c:230-245, ddt_test.c:497-503",
        "blocks": [[0, 1], [8, 8]], "extent": 16, "size": 9, "count": 4500,
        "chunks": [12],
    })
    # vector(2, 2, 5) of MPI_DOUBLE (ddt_lib.c:248-257)
    types.append({
        "name": "twice_two_doubles", "ref": "ddt_lib.c:248-257, ddt_test.c:506-512",
        "blocks": [[0, 16], [40, 16]], "extent": 56, "size": 32, "count": 4500,
        "chunks": [12],
    })
    # struct { int, double } (BASELINE config 3)
    types.append({
        "name": "struct_int_double", "ref": "BASELINE.md §4 config 3",
        "blocks": [[0, 4], [8, 8]], "extent": 16, "size": 12, "count": 1000,
        "chunks": [12, 64 * 1024],
    })
    return {"types": types}


def unpack_ooo():
    """unpack_ooo.c's fixture.  N = 331 elements (:27).  struct foo_t {int
    i[3]; double d[3];} puts i at 0/4/8 and d at 16/24/32 (extent 40); the
    type is struct{vector(2,1,2,MPI_INT) at &foo.i[0], vector(2,1,2,
    MPI_DOUBLE) at &foo.d[0]} (:167-266), so each element's typemap is
    i[0], i[2], d[0], d[2]: 24 bytes packed, the layout of struct pfoo_t
    {int i[2]; double d[2];} (:35-38)."""
    n = 331
    pbar = np.zeros(n, dtype=[("i", "<i4", 2), ("d", "<f8", 2)])
    j = np.arange(n)
    pbar["i"][:, 0] = 123 + j          # :81-84
    pbar["i"][:, 1] = 789 + j
    pbar["d"][:, 0] = 123.456 + j
    pbar["d"][:, 1] = 789.123 + j
    foo = np.dtype({"names": ["i", "pad", "d"], "formats": [("<i4", 3), "<u4", ("<f8", 3)],
                    "offsets": [0, 12, 16], "itemsize": 40})
    bar = np.zeros(n, dtype=foo)
    raw = bar.view(np.uint8).reshape(n, 40)
    for off, ln in ((0, 4), (8, 4), (16, 8), (32, 8)):   # :85-91: 0xFF over the data fields
        raw[:, off:off + ln] = 0xFF
    bar["i"][:, 1] = 0
    bar["d"][:, 1] = 0.0
    bar["pad"] = 0x5A5A5A5A  # malloc'd padding in the reference: here a pattern that must survive
    exp = bar.copy()
    exp["i"][:, 0] = pbar["i"][:, 0]   # :125-131
    exp["i"][:, 2] = pbar["i"][:, 1]
    exp["d"][:, 0] = pbar["d"][:, 0]
    exp["d"][:, 2] = pbar["d"][:, 1]
    tables = {  # :199-250
        "test1": [[992, 0], [1325, 992], [992, 2317], [992, 3309], [992, 4301], [992, 5293],
                  [992, 6285], [667, 7277]],
        "test2": [[992, 0], [992, 2317], [992, 3309], [992, 4301], [992, 5293], [992, 6285],
                  [1325, 992], [667, 7277]],
        "test3": [[992, 0], [4960, 2317], [1325, 992], [667, 7277]],
        "test4": [[992, 0], [992, 2976], [992, 1984], [992, 992], [3976, 3968]],
    }
    return {"ref": "test/datatype/unpack_ooo.c", "count": n, "extent": 40, "size": 24,
            "blocks": [[0, 4], [8, 4], [16, 8], [32, 8]],
            "desc": ["E 6 2 1 8 0", "E 16 2 1 16 16"],
            "tables": tables,
            "packed_hex": pbar.tobytes().hex(),
            "bar_init_hex": bar.tobytes().hex(),
            "expected_hex": exp.tobytes().hex()}


def main():
    for name, fn in (("op_kat.json", op_kat), ("op_edge.json", op_edge),
                     ("ring_closed_form.json", ring_closed_form), ("ddt_kat.json", ddt_kat),
                     ("unpack_ooo.json", unpack_ooo)):
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(fn(), f, indent=1, sort_keys=True)
            f.write("\n")
        print("wrote", name)


if __name__ == "__main__":
    main()
