"""The native CLI (`anx`, C++) and launcher (`anxrun`): the reference's per-version executables.
CPU versions run here; GPU versions are marked. Outputs must match the Python package bit for bit
(same C++ kernels, same counter-based RNG) — CRC-32 checksums are compared."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "cuda-mpi-gpu-cluster-programming_amd", "bin")
ANX, ANXRUN = os.path.join(BIN, "anx"), os.path.join(BIN, "anxrun")

pytestmark = pytest.mark.skipif(not os.path.exists(ANX), reason="native CLI not built")


def native(args, np_=None, timeout=300, env=None, expect=0):
    cmd = ([ANXRUN, "-np", str(np_), "--timeout", str(timeout), ANX] if np_ else [ANX]) + args
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout + 30,
                         env=dict(os.environ, OMP_NUM_THREADS="1", **(env or {})))
    ok = out.returncode != 0 if expect == "nonzero" else out.returncode == expect
    assert ok, f"rc={out.returncode}\n" + out.stdout[-2000:] + out.stderr[-3000:]
    recs = [json.loads(l[len("ANX_JSON "):]) for l in out.stdout.splitlines() if l.startswith("ANX_JSON ")]
    return (recs[0] if recs else None), out


@pytest.fixture(scope="module")
def py_serial():
    sys.path.insert(0, ROOT)
    from anx.versions import RunConfig, run
    return run(RunConfig(version="v1", init="rand", seed=3, batch=2, quiet=True)).checksum


def test_v1_golden_and_contract():
    rec, out = native(["--version", "v1"])
    assert "AlexNet Serial Forward Pass completed in" in out.stdout
    assert "44.4152 42.4612 40.6967" in out.stdout
    assert rec["shape"] == [13, 13, 256] and rec["native"] is True


def test_v1_matches_python(py_serial):
    rec, _ = native(["--version", "v1", "--init", "rand", "--seed", "3", "--batch", "2", "--check"])
    assert rec["checksum"] == py_serial
    assert rec["max_abs_err"] == 0.0


@pytest.mark.parametrize("np_", [2, 3])
def test_v21(py_serial, np_):
    rec, out = native(["--version", "v2.1", "--init", "rand", "--seed", "3", "--batch", "2"], np_)
    assert rec["np"] == np_ and rec["checksum"] == py_serial
    assert "Execution Time:" in out.stdout


@pytest.mark.parametrize("np_", [2, 4, 7])
@pytest.mark.parametrize("decomp", ["overlap", "per_layer"])
def test_v22(py_serial, np_, decomp):
    """overlap: one exact input halo per rank; per_layer: the reference's two exchanges (input rows,
    then pool1 rows after stage 1, M10 + M11). Both bit-identical to V1."""
    rec, out = native(["--version", "v2.2", "--init", "rand", "--seed", "3", "--batch", "2", "--iters", "1",
                       "--decomp", decomp], np_)
    assert rec["checksum"] == py_serial and "shape: 13x13x256" in out.stdout
    assert set(rec["phases_warm"]) >= {"scatter", "halo", "compute", "gather"}
    assert ("halo_p1" in rec["phases_warm"]) == (decomp == "per_layer")


def test_fail_stop_exit():
    """A rank that dies takes the job down (MPI_Abort semantics), nonzero exit, no hang."""
    _, out = native(["--version", "v2.2"], 3, timeout=60, env={"ANX_FAULT": "exit:1"}, expect="nonzero")
    assert "injected fault" in out.stderr


def test_fail_stop_hang_watchdog():
    """A stalled rank trips the comm watchdog of its peers (ANX_COMM_TIMEOUT) -> abort."""
    _, out = native(["--version", "v2.2"], 2, timeout=60, env={"ANX_FAULT": "hang:1", "ANX_COMM_TIMEOUT": "3"},
                    expect="nonzero")
    assert "timeout" in out.stderr


@pytest.mark.gpu
def test_native_v3_gpu(cuda):
    rec, out = native(["--version", "v3", "--iters", "3"])
    line = next(l for l in out.stdout.splitlines() if l.startswith("Final Output (first 10 values):"))
    vals = [float(v) for v in line.split(":")[1].split()[:3]]
    assert vals == pytest.approx([29.2932, 25.9153, 23.3255], abs=1e-3)  # log vs fp64: see test_gpu_engine
    assert rec["warm_ms"] is not None


@pytest.mark.gpu
def test_native_v3_batch_check(cuda):
    rec, _ = native(["--version", "v3", "--batch", "32", "--init", "rand", "--check", "--iters", "2"])
    assert rec["max_abs_err"] < 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("np_", [2, 3])
def test_native_v4_shared_gpu(cuda, np_):
    # direct conv1/conv2: every decomposition is bit-identical to the single-GPU run
    d = ["--conv2-algo", "direct", "--conv1-algo", "direct"]
    ref, _ = native(["--version", "v3", "--init", "rand", "--seed", "5", "--batch", "3", *d])
    rec, out = native(["--version", "v4", "--init", "rand", "--seed", "5", "--batch", "3", "--iters", "2", *d], np_)
    assert "Final Output Shape: 13x13x256" in out.stdout
    assert rec["checksum"] == ref["checksum"]
    # per-layer: pool1 halo rows device-staged (D2H -> host channel -> H2D) between stage 1 and 2
    rec, _ = native(["--version", "v4", "--init", "rand", "--seed", "5", "--batch", "3", "--iters", "2",
                     "--decomp", "per_layer", *d], np_)
    assert rec["checksum"] == ref["checksum"] and "halo_p1" in rec["phases_warm"]
    # Winograd conv2 (default): tile origins move with the row split -> equal to ~1e-7, not bitwise
    rec, _ = native(["--version", "v4", "--init", "rand", "--seed", "5", "--batch", "3", "--check"], np_)
    assert rec["max_abs_err"] < 1e-3


def _schedule(np_, transport, split, batch=3, decomp="per_layer", src="root"):
    _, out = native(["--version", "v5", "--dry-run", "--transport", transport, "--split", split, "--batch",
                     str(batch), "--decomp", decomp, "--input-source", src], np_)
    return sorted(l.split(" ", 2)[2] for l in out.stdout.splitlines() if l.startswith("ANX_SCHEDULE "))


@pytest.mark.parametrize("np_,split", [(2, "rows"), (3, "rows"), (4, "rows"), (4, "hybrid"), (3, "batch")])
@pytest.mark.parametrize("src", ["root", "local"])
def test_v5_transports_issue_identical_transfers(np_, split, src):
    """The RCCL, loopback and peer transports execute the same transfer list (record-only dry run:
    each logs every transfer at the point it would issue it), so the shared-GPU peer / loopback tests
    cover the RCCL schedule. Device-resident (local) input moves no scatter inside a step."""
    rccl, peer = _schedule(np_, "rccl", split, src=src), _schedule(np_, "peer", split, src=src)
    assert rccl == peer == _schedule(np_, "loopback", split, src=src) and len(rccl) > 0
    phases = {l.split(" ")[2].split("#")[0] for l in rccl}
    assert "gather" in phases and ("scatter" in phases) == (src == "root")
    assert ("halo_p1" in phases) == (split == "rows" or np_ > 3)


def test_v5_explicit_row_ways():
    """--row-ways R: R ranks per row group (4 ranks, 2-way rows = 2 groups, halos inside each group);
    it must divide the rank count."""
    _, out = native(["--version", "v5", "--dry-run", "--transport", "peer", "--row-ways", "2", "--batch", "8",
                     "--input-source", "local"], 4)
    halos = [l for l in out.stdout.splitlines() if l.startswith("ANX_SCHEDULE ") and " halo_p1" in l]
    pairs = {tuple(sorted(int(t) for t in l.split(" ")[5].split("->"))) for l in halos}
    assert pairs and pairs <= {(0, 1), (2, 3)}
    native(["--version", "v5", "--dry-run", "--row-ways", "3", "--batch", "8"], 4, expect="nonzero")


@pytest.mark.gpu
@pytest.mark.parametrize("np_,decomp,split,extra", [(2, "per_layer", "rows", []), (3, "per_layer", "rows", []),
                                                    (4, "per_layer", "rows", ["--chunks", "2"]),
                                                    (2, "overlap", "rows", []),
                                                    (4, "per_layer", "auto", ["--peer-sync", "notes"]),
                                                    (4, "per_layer", "hybrid", []), (3, "per_layer", "batch", [])])
def test_native_v5_peer_transport(cuda, np_, decomp, split, extra):
    """V5 on the native runtime with the peer transport (one hipMemcpy2DAsync per transfer into
    IPC-mapped receiver buffers, device-side flag ordering, halo chunks on their own stream, no host
    stream sync in steady state): ranks share the box's GPU, and the output is bit-identical to the
    single-GPU run (direct convs)."""
    d = ["--conv2-algo", "direct", "--conv1-algo", "direct"]
    ref, _ = native(["--version", "v3", "--init", "rand", "--seed", "6", "--batch", "3", *d])
    # pipelined steady state (scatter / gather on a second stream) with --poison: every consumed
    # buffer is NaN-filled after use, so a step that reads or overwrites one out of order changes
    # the checksum of the last step
    for pipe in ("on", "off"):
        rec, out = native(["--version", "v5", "--transport", "peer", "--decomp", decomp, "--split", split, "--init",
                           "rand", "--seed", "6", "--batch", "3", "--iters", "4", "--lrn-alpha-mode", "raw",
                           "--pipeline", pipe, "--poison", *extra, *d], np_)
        assert set(rec["phases_warm"]) == {"scatter", "stage1", "halo_p1", "stage2", "gather", "compute"}
        assert "Final Output Shape: 13x13x256" in out.stdout or rec["shape"] == [13, 13, 256]
        assert rec["checksum"] == ref["checksum"], pipe
        assert rec["v5"]["ordering"] == ("notes" if "notes" in extra else "flags")
    # default (Winograd) convs: equal to the fp64 oracle within fp32 error
    rec, _ = native(["--version", "v5", "--transport", "peer", "--init", "rand", "--seed", "6", "--batch", "3",
                     "--check"], np_)
    assert rec["max_abs_err"] < 1e-3


@pytest.mark.gpu
def test_native_v5_single_rank(cuda):
    rec, _ = native(["--version", "v5", "--init", "rand", "--batch", "4", "--check", "--iters", "2"], 1)
    assert rec["max_abs_err"] < 1e-3


def test_multinode_emulation(py_serial):
    """Two `anxrun` instances as two "nodes" (--nnodes 2 --node-rank r, shared master port): one
    4-rank job — the reference's hostfile multi-machine run (scripts/2_final_multi_machine.sh)."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    args = ["--version", "v2.2", "--init", "rand", "--seed", "3", "--batch", "2"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    node = lambda r: subprocess.Popen(  # noqa: E731
        [ANXRUN, "-np", "2", "--nnodes", "2", "--node-rank", str(r), "--master-addr", "127.0.0.1", "--port",
         str(port), "--timeout", "120", ANX, *args], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
    n1, n0 = node(1), node(0)
    out0, err0 = n0.communicate(timeout=180)
    n1.communicate(timeout=60)
    assert n0.returncode == 0 and n1.returncode == 0, err0
    rec = json.loads(next(l for l in out0.splitlines() if l.startswith("ANX_JSON "))[9:])
    assert rec["np"] == 4 and rec["checksum"] == py_serial


def _two_nodes(args, timeout=120):
    """One 4-rank job as two 2-rank `anxrun` "nodes" on this host (--nnodes 2)."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    node = lambda r: subprocess.Popen(  # noqa: E731
        [ANXRUN, "-np", "2", "--nnodes", "2", "--node-rank", str(r), "--master-addr", "127.0.0.1", "--port",
         str(port), "--timeout", str(timeout), ANX, *args], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
        env=env)
    n1, n0 = node(1), node(0)
    out0, err0 = n0.communicate(timeout=timeout + 60)
    out1, err1 = n1.communicate(timeout=60)
    return (n0.returncode, out0, err0), (n1.returncode, out1, err1)


def test_v5_multinode_transport_choice():
    """The V5 transport is chosen per node: across nodes `auto` is RCCL (the peer transport maps IPC
    buffers and works inside one host only) and an explicit `--transport peer` fails fast with a
    clear error instead of failing inside hipIpcOpenMemHandle."""
    base = ["--version", "v5", "--dry-run", "--batch", "4", "--split", "rows", "--decomp", "per_layer"]
    (rc0, out0, err0), (rc1, out1, _) = _two_nodes(base + ["--transport", "auto"])
    assert rc0 == 0 and rc1 == 0, err0
    lines = [l for l in out0.splitlines() + out1.splitlines() if l.startswith("ANX_SCHEDULE ")]
    assert lines and all(l.split(" ")[1] == "rccl" for l in lines)
    (rc0, _, err0), (rc1, _, err1) = _two_nodes(base + ["--transport", "peer"], timeout=60)
    assert rc0 != 0 and rc1 != 0
    assert "single-node" in err0 + err1


@pytest.mark.gpu
def test_v5_rows2_transports_bitwise(cuda):
    """bench.py's V5 sub-records (2-way row groups, the pool1 halo on) per device transport: the peer
    transport and the RCCL transport's code over the loopback device comm, on ranks sharing the GPU,
    NaN-poisoned and pipelined, move the same halo bytes and give the same output bits (Winograd convs,
    the bench's kernels), and match the single-rank run to fp32 rounding."""
    args = ["--version", "v5", "--row-ways", "2", "--init", "rand", "--seed", "8", "--batch", "40", "--iters", "3",
            "--chunks", "1", "--poison", "--pipeline", "on"]
    peer, _ = native([*args, "--transport", "peer"], 2)
    loop, _ = native([*args, "--transport", "loopback"], 2)
    for r in (peer, loop):
        assert r["v5"]["halo_transfers_per_step"] > 0 and r["v5"]["halo_bytes_per_step"] > 0
        assert "none" not in r["v5"]["halo_exchange"]
    assert peer["checksum"] == loop["checksum"]
    assert peer["v5"]["halo_bytes_per_step"] == loop["v5"]["halo_bytes_per_step"]
    assert peer["v5"]["transport"] == "peer" and loop["v5"]["transport"] == "rccl-loopback"
    one, _ = native(["--version", "v5", "--init", "rand", "--seed", "8", "--batch", "40", "--check"], 1)
    two, _ = native([*args, "--transport", "peer", "--check"], 2)
    assert one["max_abs_err"] < 1e-3 and two["max_abs_err"] < 1e-3
