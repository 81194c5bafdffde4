"""The MCA glue compiled against the reference's own framework headers
(VERDICT r3 item 7), `gcc -fsyntax-only -Wall -Wextra`: coll/rocm, pml/rocm,
osc/rocm, op/rocm and the convertor seam (with OPAL_CUDA_SUPPORT 0 and 1)
against /root/reference's ompi/mca/coll/coll.h, ompi/mca/pml/pml.h,
ompi/mca/osc/osc.h, ompi/mca/op/op.h, opal/datatype/*.h, communicator.h,
request.h ... as they are.  Only what configure generates is stood in for
(tests/realhdr/: opal_config.h, libevent's event-config.h, and mpi.h made
from mpi.h.in into a scratch directory by tests/realhdr/gen_mpi_h.py), plus
type names of the two third-party libraries whose submodules are empty
(pmix, hwloc).  CPU only; skipped where the reference is not present (the
GPU box)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
HERE = os.path.join(ROOT, "tests", "realhdr")

pytestmark = pytest.mark.skipif(not os.path.isfile(os.path.join(REF, "ompi/include/mpi.h.in")),
                                reason="the reference tree is not present here")

GLUE = [("coll/rocm/coll_rocm_module.c", None), ("pml/rocm/pml_rocm.c", None),
        ("osc/rocm/osc_rocm_component.c", None), ("op/rocm/op_rocm_component.c", None),
        ("common/rocm/opal_datatype_rocm.c", 0), ("common/rocm/opal_datatype_rocm.c", 1)]


@pytest.fixture(scope="module")
def config_dirs(tmp_path_factory):
    import sys
    sys.path.insert(0, HERE)
    from gen_mpi_h import generate
    dirs = {}
    for cuda in (0, 1):
        d = tmp_path_factory.mktemp(f"cfg{cuda}")
        generate(os.path.join(REF, "ompi/include/mpi.h.in"), str(d / "mpi.h"))
        cfg = open(os.path.join(HERE, "opal_config.h")).read()
        (d / "opal_config.h").write_text(cfg.replace("#define OPAL_CUDA_SUPPORT 0",
                                                     f"#define OPAL_CUDA_SUPPORT {cuda}"))
        dirs[cuda] = str(d)
    return dirs


@pytest.mark.parametrize("src,cuda", GLUE, ids=[f"{s.split('/')[-1]}{'' if c is None else f'-cuda{c}'}"
                                                for s, c in GLUE])
def test_glue_compiles_against_reference_headers(config_dirs, src, cuda):
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    path = os.path.join(ROOT, "ompi_amd", "mca", src)
    cmd = ["gcc", "-fsyntax-only", "-std=gnu11", "-Wall", "-Wextra", "-Wno-unused-parameter",
           "-Wno-missing-field-initializers", "-Wno-sign-compare",
           "-I", config_dirs[cuda or 0], "-I", HERE, "-I", REF, "-I", os.path.join(REF, "opal/include"),
           "-I", os.path.join(REF, "ompi/include"),
           "-I", os.path.join(REF, "opal/mca/event/libevent2022/libevent"),
           "-I", os.path.join(REF, "opal/mca/event/libevent2022/libevent/include"),
           "-I", os.path.join(ROOT, "include"), "-I", os.path.dirname(path), path]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    ours = [ln for ln in r.stderr.splitlines()
            if ("error" in ln or "warning" in ln) and not ln.startswith(REF)]
    assert r.returncode == 0 and not ours, (r.returncode, "\n".join(ours) or r.stderr[-3000:])
