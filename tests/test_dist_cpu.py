"""Multi-process tests of the distributed paths on CPU ranks over gloo (world_size 2 and 4).

The reference "tested" distribution only by eyeballing mpirun --oversubscribe output;
these assert that every decomposition returns exactly the single-process result.
"""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _pipeline_worker(rank, world, port, q, prefetch=False):
    sys.path.insert(0, ROOT)
    import anx  # noqa: F401
    from anx.models.alexnet_blocks import AlexNetBlocks
    from anx.parallel.pipeline import PipelineConfig, ScatterComputeGather
    from anx.utils.init import init_input
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    d = anx.blocks_dims()
    m = AlexNetBlocks(init="rand", seed=2, device="cpu")
    pipe = ScatterComputeGather(m, PipelineConfig(2, micro=2, prefetch=prefetch), (d.H, d.W, d.C0),
                                (d.Hp2, d.Wp2, d.C2), "cpu")
    if rank == 0:
        pipe.x_global.copy_(init_input(2 * world, "rand", seed=2).view(world, 2, d.H, d.W, d.C0))
    for _ in range(3 if prefetch else 1):
        pipe.step()
    pipe.drain()
    if rank == 0:
        q.put(pipe.y_global.clone())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("prefetch", [False, True])
def test_scatter_compute_gather_gloo(prefetch):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_pipeline_worker, args=(r, world, port, q, prefetch)) for r in range(world)]
    for p in procs:
        p.start()
    y = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    sys.path.insert(0, ROOT)
    from anx.models.alexnet_blocks import AlexNetBlocks
    from anx.utils.init import init_input
    m = AlexNetBlocks(init="rand", seed=2, device="cpu")
    ref = m(init_input(2 * world, "rand", seed=2))
    torch.testing.assert_close(y.view_as(ref), ref, rtol=0, atol=0)


def _async_lanes_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import anx  # noqa: F401
    from anx.models.alexnet_blocks import AlexNetBlocks
    from anx.parallel.pipeline import PipelineConfig, ScatterComputeGather
    from anx.utils.init import init_input
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    d = anx.blocks_dims()
    m = AlexNetBlocks(init="rand", seed=2, device="cpu")
    pipe = ScatterComputeGather(m, PipelineConfig(2, scatter=False, prefetch=True, async_lanes=True),
                                (d.H, d.W, d.C0), (d.Hp2, d.Wp2, d.C2), "cpu")
    assert pipe.async_lanes and len(pipe._yb) == 2
    pipe._xb[0].copy_(init_input(2 * world, "rand", seed=2)[2 * rank:2 * rank + 2])
    for _ in range(3):  # per-lane gathers; a step waits for the gather that read its buffer 2 steps ago
        pipe.step()
    pipe.drain()
    if rank == 0:
        q.put(pipe.y_global.clone())
    dist.barrier()
    dist.destroy_process_group()


def test_async_lanes_pipeline_gloo():
    """The bench's default dp step (local input, free-running lanes with per-lane gathers: the
    model's forward_async; on CPU ranks one lane) gathers exactly the single-process outputs."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_async_lanes_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    y = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    sys.path.insert(0, ROOT)
    from anx.models.alexnet_blocks import AlexNetBlocks
    from anx.utils.init import init_input
    m = AlexNetBlocks(init="rand", seed=2, device="cpu")
    ref = m(init_input(2 * world, "rand", seed=2))
    torch.testing.assert_close(y.view_as(ref), ref, rtol=0, atol=0)


def _shed_worker(rank, world, port, q, mode):
    sys.path.insert(0, ROOT)
    import anx  # noqa: F401
    from anx.models.alexnet_blocks import AlexNetBlocks
    from anx.parallel.pipeline import PipelineConfig, ScatterComputeGather
    from anx.utils.init import init_input
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    d = anx.blocks_dims()
    m = AlexNetBlocks(init="rand", seed=2, device="cpu")
    cfg = PipelineConfig(2, micro=1, scatter=False, prefetch=mode != "plain", async_lanes=mode == "async", root_batch=1)
    pipe = ScatterComputeGather(m, cfg, (d.H, d.W, d.C0), (d.Hp2, d.Wp2, d.C2), "cpu")
    assert pipe.shed and pipe.x.shape[0] == (1 if rank == 0 else 2)
    xs = init_input(2 * world, "rand", seed=2)
    for xb in pipe._xb:
        xb.copy_(xs[2 * rank:2 * rank + pipe.x.shape[0]])
    for _ in range(3):
        pipe.step()
    pipe.drain()
    if rank == 0:
        q.put(pipe.y_global.clone())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["async", "prefetch", "plain"])
def test_root_batch_shed_gloo(mode):
    """dp with rank 0 shedding images (root_batch < batch_per_rank): the point-to-point gather puts
    every peer's full batch and the root's smaller one where the single-process result has them."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_shed_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    y = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    sys.path.insert(0, ROOT)
    from anx.models.alexnet_blocks import AlexNetBlocks
    from anx.utils.init import init_input
    m = AlexNetBlocks(init="rand", seed=2, device="cpu")
    ref = m(init_input(2 * world, "rand", seed=2)).view(world, 2, *y.shape[2:])
    torch.testing.assert_close(y[0, :1], ref[0, :1], rtol=0, atol=0)
    torch.testing.assert_close(y[1:], ref[1:], rtol=0, atol=0)


def _shed_reject_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import anx  # noqa: F401
    from anx.models.alexnet_blocks import AlexNetBlocks
    from anx.parallel.pipeline import PipelineConfig, ScatterComputeGather
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d = anx.blocks_dims()
    m = AlexNetBlocks(init="rand", seed=2, device="cpu")
    errs = []
    for cfg in (PipelineConfig(2, scatter=True, root_batch=1),     # the root's input is scattered
                PipelineConfig(4, micro=2, scatter=False, root_batch=1),  # fewer micro-batches on the root
                PipelineConfig(2, scatter=False, root_batch=3)):  # more than a peer's batch
        try:
            ScatterComputeGather(m, cfg, (d.H, d.W, d.C0), (d.Hp2, d.Wp2, d.C2), "cpu")
            errs.append(None)
        except ValueError as e:
            errs.append(str(e))
    q.put(errs)
    dist.barrier()
    dist.destroy_process_group()


def test_root_batch_rejects_unsupported_shapes():
    """root_batch needs local input, the peers' micro-batch count and at most a peer's batch."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_shed_reject_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    errs = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for e in errs:
        assert all(x is not None for x in e), e


def _prefetch_changing_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import anx  # noqa: F401
    from anx.models.alexnet_blocks import AlexNetBlocks
    from anx.parallel.pipeline import PipelineConfig, ScatterComputeGather
    from anx.utils.init import init_input
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    d = anx.blocks_dims()
    m = AlexNetBlocks(init="rand", seed=2, device="cpu")
    pipe = ScatterComputeGather(m, PipelineConfig(1, micro=1, prefetch=True), (d.H, d.W, d.C0),
                                (d.Hp2, d.Wp2, d.C2), "cpu")
    outs = []
    for k in range(4):  # a new batch written into x_global after every step
        if rank == 0:
            pipe.x_global.copy_(init_input(world, "rand", seed=10 + k).view(world, 1, d.H, d.W, d.C0))
        pipe.step()
        pipe.drain()
        if rank == 0:
            outs.append(pipe.y_global.clone())
    if rank == 0:
        q.put(torch.stack(outs))
    dist.barrier()
    dist.destroy_process_group()


def test_prefetch_pipeline_input_semantics():
    """With prefetch, step k computes the batch x_global held when step k-1 was called (step 0 its
    own): inputs rewritten between steps are never mixed or lost."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_prefetch_changing_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    ys = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    sys.path.insert(0, ROOT)
    from anx.models.alexnet_blocks import AlexNetBlocks
    from anx.utils.init import init_input
    m = AlexNetBlocks(init="rand", seed=2, device="cpu")
    for k in range(4):
        src = max(k - 1, 0)
        ref = m(init_input(world, "rand", seed=10 + src))
        torch.testing.assert_close(ys[k].view_as(ref), ref, rtol=0, atol=0)


def _workload_worker(rank, world, port, q, version, decomp, batch, root_images=-1):
    sys.path.insert(0, ROOT)
    import anx  # noqa: F401
    from anx.parallel.workloads import NativeV5
    from anx.utils.init import init_input, init_weights
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    kw = dict(layer="overlap", input_source="root") if version == "v4" else dict(layer="per_layer")
    wl = NativeV5(batch, init_weights("rand", 4) if rank == 0 else None, decomp=decomp, impl="host",
                  timeout_s=120, keep_log=True, root_images=root_images, **kw)
    wl.fill(init_input(batch, "rand", seed=4) if rank == 0 else None)
    wl.step()
    wl.step()  # steady state: the other parity's buffers
    d = wl.describe()
    assert d["transport"] == "host" and d["device"] == -1
    log = wl.transfer_log()
    if rank == 0:
        q.put((wl.output().clone(), d, len(log)))
    wl.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("version,decomp,world,batch", [
    ("v5", "rows", 2, 2), ("v5", "rows", 3, 1), ("v5", "hybrid", 4, 3), ("v4", "rows", 2, 2),
    ("v4", "hybrid", 3, 2), ("v5", "batch", 2, 3), ("v5", "rows2", 4, 2)])
def test_native_v5_host_gloo(version, decomp, world, batch):
    """The native V5 runtime in host mode (CPU ranks: host engine, host transport; the same layout,
    schedule and halo chunks as on GPUs, libanx_dist) reproduces the single-process output bit for
    bit: V5 per_layer tiles with the pool1 halo exchange, and V4's overlap tiles scattered from the root
    every step."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_workload_worker, args=(r, world, port, q, version, decomp, batch))
             for r in range(world)]
    for p in procs:
        p.start()
    y, d, nlog = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    sys.path.insert(0, ROOT)
    from anx.models.alexnet_blocks import AlexNetBlocks
    from anx.utils.init import init_input
    ref = AlexNetBlocks(init="rand", seed=4, device="cpu")(init_input(batch, "rand", seed=4))
    torch.testing.assert_close(y.view_as(ref), ref, rtol=0, atol=0)
    assert d["decomp"] == ("overlap" if version == "v4" else "per_layer")
    assert d["input_source"] == ("root" if version == "v4" else "local")
    assert nlog > 0


def test_native_v5_host_root_shedding_gloo():
    """The dp program with root shedding in the native runtime, host mode: rank 0
    computes 1 image, the two peers 3 each, gathered to rank 0 -- bit for bit the single-process output."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_workload_worker, args=(r, 3, port, q, "v5", "batch", 7, 1)) for r in range(3)]
    for p in procs:
        p.start()
    y, d, nlog = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    sys.path.insert(0, ROOT)
    from anx.models.alexnet_blocks import AlexNetBlocks
    from anx.utils.init import init_input
    ref = AlexNetBlocks(init="rand", seed=4, device="cpu")(init_input(7, "rand", seed=4))
    torch.testing.assert_close(y.view_as(ref), ref, rtol=0, atol=0)
    assert d["images_per_rank"] == [1, 3, 3] and d["row_ways"] == 1
    assert d["halo_exchange"].startswith("none")


@pytest.mark.parametrize("workload", ["v4", "v5"])
def test_bench_workload_contract_gloo(workload):
    """bench.py --workload v4|v5 at N=2 (gloo/CPU rehearsal): one JSON line, strong scaling, phases."""
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--steps", "1", "--warmup", "0", "--workload", workload, "--batch", "2", "--device", "cpu"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["scaling"] == "strong" and rec["config"]["global_batch"] == 2 and rec["value"] > 0
    assert rec["config"]["workload"] == workload and rec["config"]["parallelism"] == f"{workload}-rows2"


def test_bench_contract_gloo():
    """bench.py under torch.distributed.run (gloo/CPU rehearsal) prints ONE valid JSON line on rank 0."""
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--steps", "1", "--warmup", "0", "--batch-per-gpu", "2", "--micro", "2", "--device", "cpu",
           "--no-ref-programs"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in rec
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == 4 and rec["value"] > 0


def test_bench_root_batch_gloo():
    """bench.py --root-batch (gloo/CPU rehearsal): the JSON counts the root's shed share in the job."""
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--steps", "1", "--warmup", "0", "--batch-per-gpu", "2", "--root-batch", "1", "--device", "cpu",
           "--no-ref-programs"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert rec["config"]["global_batch"] == 3 and rec["config"]["root_batch"] == 1
    assert rec["config"]["batch_per_gpu"] == 2


def _bench3(extra_env=None, extra_args=()):
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"), "--gpus", "3",
           "--steps", "1", "--warmup", "0", "--batch-per-gpu", "4", "--root-batch", "2", "--device", "cpu",
           "--no-ref-programs", *extra_args]
    env = dict(os.environ, OMP_NUM_THREADS="1", **(extra_env or {}))
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def test_bench_selfcheck_gloo_n3():
    """The N>1 record proves itself (gloo/CPU rehearsal at N=3): the communicator's world size and every
    rank's identity; rank 0's share calibrated from measured per-rank compute spans (modelled / forced
    value and the calibration rounds both reported); one post-window step whose gathered outputs match
    every rank's own checksum, and two images per rank against the fp64 oracle."""
    rec = _bench3(extra_args=("--calibrate-root", "on"))
    assert rec["rccl_world_size"] == 3
    ident = rec["identity"]
    assert ident["world_size"] == 3 and [r["rank"] for r in ident["ranks"]] == [0, 1, 2]
    assert ident["backend"] == "gloo"
    cfg = rec["config"]
    assert cfg["root_batch_modelled"] == 2 and "calibrated_root_batch" in cfg and cfg["calibration"]
    assert 1 <= cfg["root_batch"] <= 4 and cfg["global_batch"] == 2 * 4 + cfg["root_batch"]
    assert rec["gather_verified"] is True and rec["verify"]["mismatched_ranks"] == []
    assert [r["images"] for r in rec["verify"]["per_rank"]] == [cfg["root_batch"], 4, 4]
    assert rec["verify"]["oracle_max_rel_err"] < 1e-5


def test_bench_selfcheck_detects_corrupt_rank_gloo():
    """A rank whose gathered bytes do not match what it computed turns gather_verified false and is named."""
    rec = _bench3({"ANX_BENCH_CORRUPT_RANK": "2"}, ("--calibrate-root", "off"))
    assert rec["gather_verified"] is False and rec["verify"]["mismatched_ranks"] == [2]
    assert "calibration" not in rec["config"] and rec["config"]["root_batch"] == 2


def test_bench_secondary_deadline_keeps_headline_gloo():
    """A secondary program that hangs on one rank (here rank 1 blocks where the native V4/V5 programs
    start) cannot take the measured headline with it: past --secondary-deadline-s rank 0 prints the
    headline record, marked with the pending stage, and every rank exits 0."""
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--steps", "1", "--warmup", "0", "--batch-per-gpu", "2", "--device", "cpu", "--secondary-deadline-s", "15"]
    env = dict(os.environ, OMP_NUM_THREADS="1", ANX_BENCH_HANG_STAGE="reference_programs:1")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["value"] > 0 and rec["n_gpus"] == 2 and rec["gather_verified"] is True
    assert rec["secondary_deadline"] == {"seconds": 15.0, "pending_stage": "reference_programs"}
    assert "v4" not in rec and "v5" not in rec and "secondary_s" not in rec
    assert "secondary records still running" in out.stderr


@pytest.mark.parametrize("world", [2, 3])
def test_bench_reference_programs_gloo(world):
    """The default dp run also measures BASELINE configs 3 and 4 on the same ranks:
    ``v4`` and ``v5`` secondary objects from the native runtimes (host mode on CPU ranks), V5 both at the
    cost model's pick and with the pool1 halo exchange forced on (2-way row groups; all ranks' rows at an
    odd count), each with its rate, halo bytes, halo phase and an exact output checksum; the headline
    record is unchanged and the modelled curve sits outside ``config``."""
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"), "--gpus", str(world),
           "--steps", "1", "--warmup", "0", "--batch-per-gpu", "2", "--device", "cpu", "--ref-steps", "1",
           "--ref-batch-v4", "2", "--ref-batch-v5", str(world)]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == world and rec["scaling"] == "weak" and rec["config"]["parallelism"] == f"dp{world}"
    assert rec["config"]["model"].startswith("AlexNet Blocks1-2")  # the model's name, not the modelled curve
    v4, v5 = rec["v4"], rec["v5"]
    assert v4["scaling"] == v5["scaling"] == "strong"
    a4 = v4["auto"]
    assert "error" not in a4, a4
    assert a4["global_batch"] == 2 and a4["images_per_s"] > 0 and "halo_exchange" in a4 and "output_crc" in a4
    a5 = v5["auto"]
    assert "error" not in a5, a5
    assert a5["global_batch"] == world and a5["images_per_s"] > 0 and isinstance(a5["output_crc"], int)
    halo = v5["rows2_host" if world % 2 == 0 else "rows_host"]
    assert "error" not in halo, halo
    assert halo["row_ways"] == (2 if world % 2 == 0 else world)
    assert halo["halo_exchange"].startswith("pool1 rows") and halo["halo_bytes_per_step"] > 0
    assert halo["halo_p1_ms"] is not None and isinstance(halo["output_crc"], int)
