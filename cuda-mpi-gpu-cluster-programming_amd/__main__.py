"""Command line: ``python -m anx <command>`` (or ``python anx.py``-style via the repo alias).

  run      run one staged version (v1 v2.1 v2.2 v3 v4 v5) in this process / torchrun rank
  launch   start N ranks of ``run`` on this node (the reference's ``mpirun -np N ./template``)
  plan     print the exact row decomposition for np ranks, or (--model dp|v4|v5) the modelled
           1/2/4/8-GPU scaling curve of a workload
  bench    shortcut for the headline benchmark (bench.py)
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys


def _run_args(ap):
    ap.add_argument("--version", "-v", default="v3", choices=["v1", "v2.1", "v2.2", "v3", "v4", "v5"])
    ap.add_argument("--batch", "-b", type=int, default=1)
    ap.add_argument("--init", default="const", choices=["const", "rand"])
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--lrn-alpha-mode", default=None, choices=["div_n", "raw"])
    ap.add_argument("--groups", type=int, default=1, choices=[1, 2], help="Conv2 groups (2 = AlexNet paper)")
    ap.add_argument("--decomp", default=None, choices=["overlap", "per_layer"])
    ap.add_argument("--strategy", default="rows", choices=["rows", "batch", "filter"],
                    help="multi-rank split: rows (spatial + halos), batch (images), filter (Conv2 filters, P7)")
    ap.add_argument("--iters", type=int, default=0, help="warm iterations after the cold run")
    ap.add_argument("--impl", default="mfma", choices=["mfma", "direct"])
    ap.add_argument("--conv2-algo", default="auto", choices=["auto", "direct", "winograd"])
    ap.add_argument("--conv1-algo", default="auto", choices=["auto", "direct", "winograd"],
                    help="direct = bit-identical across row decompositions (Winograd: ~1e-7)")
    ap.add_argument("--check", action="store_true", help="compare with the PyTorch fp64 oracle")
    ap.add_argument("--cpu-rehearsal", action="store_true", help="run a GPU version's program on CPU ranks")
    ap.add_argument("--quiet", action="store_true")


def cmd_run(a):
    from .versions import RunConfig, run
    cfg = RunConfig(version=a.version, batch=a.batch, init=a.init, seed=a.seed, lrn_mode=a.lrn_alpha_mode,
                    groups2=a.groups, decomp=a.decomp, strategy=a.strategy, iters=a.iters, impl=a.impl,
                    conv2_algo=a.conv2_algo, conv1_algo=a.conv1_algo,
                    check=a.check, quiet=a.quiet, cpu_rehearsal=a.cpu_rehearsal)
    run(cfg)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(np_: int, argv: list[str], timeout: float | None = None) -> int:
    """Start np ranks of ``python -m anx run <argv>`` with torch.distributed env (rendezvous on
    127.0.0.1). Returns the first nonzero exit code (fail-stop, like MPI_Abort)."""
    port = _free_port()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    procs = []
    for r in range(np_):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(np_), LOCAL_WORLD_SIZE=str(np_),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-c", "import anx.__main__ as m; m.main()", "run", *argv],
                                      env=env, cwd=root))
    rc = 0
    for p in procs:
        try:
            c = p.wait(timeout=timeout)
        except subprocess.TimeoutExpired:
            c = 124
        rc = rc or c
    if rc:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return rc


def cmd_launch(a, rest):
    raise SystemExit(launch(a.np, rest, a.timeout))


def cmd_plan(a):
    from .parallel.plan import conv1_redundancy, make_hybrid_plan, make_plan, pick_row_ways, plan_stats
    if a.model:  # the modelled 1/2/4/8-GPU curve of a workload (anx/cost.hpp; not a measurement)
        from .parallel import cost
        batch = a.batch or {"dp": 128, "v4": 256, "v5": 1024}[a.model]
        src = "root" if a.model == "v4" else a.input_source
        c = cost.curve(a.model, batch, row_ways=a.row_ways, input_source=src,
                       mode="overlap" if a.model == "v4" else a.decomp, overrides=a.cost)
        if a.json:
            print(json.dumps(c))
            return
        unit = "images per GPU (weak scaling)" if a.model == "dp" else "images in all (strong scaling)"
        print(f"MODELLED (not measured) {a.model} {batch} {unit}, input {src}:")
        print(cost.table(c))
        for st in c["steps"]:
            b = st["bytes"]
            print(f"N={st['np']}: compute {st['compute_ms']:.3f} ms, egress {st['egress_ms']:.3f}, ingress "
                  f"{st['ingress_ms']:.3f}, halo {st['halo_ms']:.3f} (exposed {st['halo_exposed_ms']:.3f}), h2d "
                  f"{st['h2d_ms']:.3f}; root egress {b['root_egress'] / 1e6:.1f} MB, root ingress "
                  f"{b['root_ingress'] / 1e6:.1f} MB, max rank h2d {b['max_rank_h2d'] / 1e6:.1f} MB, max rank halo "
                  f"{b['max_rank_halo'] / 1e6:.2f} MB")
        p = c["params"]
        print(f"params: xGMI {p['xgmi_gbps']} GB/s per link (assumed), H2D {p['h2d_gbps']} GB/s (measured), "
              f"host {p['host_gbps']} GB/s (assumed), root ingest slowdown {p['ingest_slowdown']}")
        return
    if a.batch is not None:  # hybrid batch x rows plan
        rw = pick_row_ways(a.np, a.batch, "v5", a.input_source, a.decomp) if a.row_ways < 0 else a.row_ways
        hp = make_hybrid_plan(227, 227, a.np, a.batch, rw, a.decomp)
        st = plan_stats(hp)
        print(f"np {a.np} batch {a.batch}: {hp.groups} group(s) of {st['row_ways']} rank(s) (row_ways {rw}"
              f"{' = the cost model pick' if a.row_ways < 0 else ''}); output rows per rank max {st['out_rows_max']} / "
              f"mean {st['out_rows_mean']:.3f}; work max/mean {st['imbalance']:.3f}; redundant conv1 rows "
              f"{100 * st['conv1_redundancy']:.1f}% of one device's")
        for r in range(a.np):
            t, im = hp.tile(r), hp.images_of(r)
            print(f"rank {r}: group {hp.group_of[r]} ({hp.group_size[hp.group_of[r]]} ranks) images "
                  f"{im.lo}..{im.hi - 1}  out rows {t.out.lo}..{t.out.hi - 1}  input rows {t.inp.lo}..{t.inp.hi - 1}")
        return
    p = make_plan(227, 227, a.np, a.decomp)
    print(f"redundant conv1 rows: {100 * conv1_redundancy(p):.1f}% of one device's")
    for r, t in enumerate(p.tiles):
        print(f"rank {r}: out {t.out.lo}..{t.out.hi - 1}  pool1 {t.p1.lo}..{t.p1.hi - 1}  conv1 {t.c1.lo}..{t.c1.hi - 1}"
              f"  input {t.inp.lo}..{t.inp.hi - 1}  owned input {p.owned_in[r].lo}..{p.owned_in[r].hi - 1}")
    for x in p.in_halos:
        print(f"input halo rows {x.rows.lo}..{x.rows.hi - 1}: rank {x.src} -> {x.dst}")
    for x in p.p1_halos:
        print(f"pool1 halo rows {x.rows.lo}..{x.rows.hi - 1}: rank {x.src} -> {x.dst}")


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser(prog="anx")
    sub = ap.add_subparsers(dest="cmd", required=True)
    _run_args(sub.add_parser("run"))
    lp = sub.add_parser("launch")
    lp.add_argument("--np", "-n", type=int, required=True)
    lp.add_argument("--timeout", type=float, default=None)
    pp = sub.add_parser("plan")
    pp.add_argument("--np", "-n", type=int, default=4)
    pp.add_argument("--decomp", default="overlap", choices=["overlap", "per_layer"])
    pp.add_argument("--batch", "-b", type=int, default=None, help="hybrid batch x rows plan for this many images")
    pp.add_argument("--row-ways", type=int, default=-1,
                    help="ranks per image group (-1 = the V4/V5 runtimes' default: the cost model's pick, 0 = batch first)")
    pp.add_argument("--model", default=None, choices=["dp", "v4", "v5"],
                    help="print the MODELLED 1/2/4/8-GPU scaling curve of a workload (anx/cost.hpp)")
    pp.add_argument("--input-source", default="local", choices=["local", "root"],
                    help="v5 / dp input: device-resident (local) or scattered by the root every step")
    pp.add_argument("--cost", default="", help="cost-model overrides, name=value;... (e.g. xgmi_gbps=64)")
    pp.add_argument("--json", action="store_true", help="--model: print the curve as JSON")
    sub.add_parser("bench")
    if argv and argv[0] == "launch":
        a, rest = ap.parse_known_args(argv)
        if rest and rest[0] == "--":
            rest = rest[1:]
        return cmd_launch(a, rest)
    if argv and argv[0] == "bench":
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        raise SystemExit(subprocess.call([sys.executable, os.path.join(root, "bench.py"), *argv[1:]]))
    a = ap.parse_args(argv)
    {"run": cmd_run, "plan": cmd_plan}[a.cmd](a)


if __name__ == "__main__":
    main()
