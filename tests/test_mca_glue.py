"""The op component glue (ompi_amd/mca/op/rocm) driven through the op
framework's selection protocol (op_base_op_select.c:90-211) by
tests/mca_harness: slot ownership, the NULL-pattern check, host-buffer
fallback to op/base (CPU) and the device path (GPU)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    from ompi_amd import _lib
    from oracle import oracle as orc
    _lib.load()
    orc.lib()
    out = str(tmp_path_factory.mktemp("mca") / "op_select_harness")
    subprocess.run(["bash", os.path.join(ROOT, "tests", "mca_harness", "build.sh"), out], check=True)
    return out


def test_op_component_selection_and_host_fallback(harness):
    r = subprocess.run([harness], capture_output=True, text=True, timeout=120,
                       env={**os.environ, "HARNESS_GPU": "0"})
    assert r.returncode == 0 and r.stdout.strip() == "ok", (r.stdout, r.stderr)


@pytest.mark.gpu
def test_op_component_device_path(harness):
    r = subprocess.run([harness], capture_output=True, text=True, timeout=120,
                       env={**os.environ, "HARNESS_GPU": "1"})
    assert r.returncode == 0 and r.stdout.strip() == "ok gpu", (r.stdout, r.stderr)
