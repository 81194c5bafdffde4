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


# ---- coll/rocm (ompi_amd/mca/coll/rocm) through tests/mca_harness/coll_harness.c ----

@pytest.fixture(scope="module")
def coll_harness(tmp_path_factory):
    from ompi_amd import _lib
    from oracle import oracle as orc
    _lib.load()
    orc.lib()
    out = str(tmp_path_factory.mktemp("mca") / "coll_harness")
    subprocess.run(["bash", os.path.join(ROOT, "tests", "mca_harness", "build_coll.sh"), out],
                   check=True)
    return out


def _run_coll_harness(exe, n, gpu, timeout):
    import secrets
    name = secrets.token_hex(3)
    env = {**os.environ, "HARNESS_GPU": "1" if gpu else "0", "HSA_ENABLE_IPC_MODE_LEGACY": "0",
           "OMPI_AMD_COLL_TIMEOUT_MS": "20000"}
    procs = [subprocess.Popen([exe, name, str(r), str(n)], stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True, env=env) for r in range(n)]
    outs = []
    try:
        for p in procs:
            out, err = p.communicate(timeout=timeout)
            outs.append((p.returncode, out.strip(), err[-2000:]))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return outs


def test_coll_component_selection(coll_harness):
    """comm_query accepts node-local intra-communicators of 2..16 ranks;
    init_query refuses without a device (coll_base_comm_select.c protocol)."""
    for rc, out, err in _run_coll_harness(coll_harness, 2, False, 60):
        assert rc == 0 and out == "ok", (rc, out, err)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 3])
def test_coll_component_device_path(coll_harness, n):
    """enable saves/retains the previous functions; every collective called
    through the communicator's table runs on device buffers and matches the
    oracle bit for bit; host / mixed / user-op calls go to the saved
    functions on every rank; release destroys the device communicator."""
    for rc, out, err in _run_coll_harness(coll_harness, n, True, 240):
        assert rc == 0 and out == "ok gpu", (rc, out, err)


# ---- osc/rocm (ompi_amd/mca/osc/rocm) through tests/mca_harness/osc_harness.c ----

@pytest.fixture(scope="module")
def osc_harness(tmp_path_factory):
    from ompi_amd import _lib
    from oracle import oracle as orc
    _lib.load()
    orc.lib()
    out = str(tmp_path_factory.mktemp("mca") / "osc_harness")
    subprocess.run(["bash", os.path.join(ROOT, "tests", "mca_harness", "build_osc.sh"), out],
                   check=True)
    return out


def test_osc_component_selection(osc_harness):
    """osc_init refuses without a device; osc_query refuses host memory,
    allocate without the device info key, inter-communicators, remote peers
    and dynamic windows (ompi_osc_base_select protocol)."""
    for rc, out, err in _run_coll_harness(osc_harness, 1, False, 60):
        assert rc == 0 and out == "ok", (rc, out, err)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 3])
def test_osc_component_device_path(osc_harness, n):
    """MPI_Win_create over device memory and MPI_Win_allocate through the
    component: fence epochs with accumulate (bit-exact vs op/base) and get,
    an exclusive-lock put epoch, a fetch_and_op counter, refusal of user ops,
    mismatched datatypes and PSCW, free."""
    for rc, out, err in _run_coll_harness(osc_harness, n, True, 180):
        assert rc == 0 and out == "ok gpu", (rc, out, err)
