"""The run-log warehouse / analytics CLI (tools/log_analysis.py): ingest of every
record format (ANX_JSON, bench JSON, 20-column harness CSV, the reference's run logs, tagged), the
speedup / efficiency tables, plots, export and the synthesis report, on a synthetic log tree."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "tools", "log_analysis.py")


def cli(*args, cwd):
    r = subprocess.run([sys.executable, TOOL, *args], cwd=cwd, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def anx_json(version, np_, ms, batch=1):
    return "ANX_JSON " + json.dumps(dict(version=version, np=np_, batch=batch, warm_ms=ms, cold_ms=ms * 2, native=True,
                                         shape=[13, 13, 256], checksum=1))


@pytest.fixture()
def tree(tmp_path):
    ours = tmp_path / "ours"
    ours.mkdir()
    (ours / "run_a.log").write_text("\n".join([anx_json("v1", 1, 40.0), anx_json("v2.2", 1, 40.0),
                                               anx_json("v2.2", 2, 25.0), anx_json("v2.2", 4, 16.0),
                                               anx_json("v3", 1, 0.2)]))
    (ours / "bench.log").write_text(json.dumps({"metric": "m", "value": 190000.0, "n_gpus": 1, "ms_per_step": 0.67,
                                                "config": {"parallelism": "dp1", "global_batch": 128}}))
    ref = tmp_path / "ref" / "logs"
    ref.mkdir(parents=True)
    (ref / "run_v1_np1.log").write_text("AlexNet V1 completed in 600.0 ms\n")
    (ref / "run_v3_np1.log").write_text("Execution Time: 200.0 ms\n")
    (ref / "summary.csv").write_text("ProjectVariant,NumProcesses,ExecutionTime_ms,OutputShape,MachineID\n"
                                     "V2.2 ScatterHalo,2,320.0,13x13x256,ref\n")
    return tmp_path


def test_ingest_speedup_report(tree):
    db = str(tree / "w.db")
    assert "ingested 6 new rows" in cli("ingest", "--root", "ours", "--db", db, cwd=tree)
    assert "ingested 3 new rows" in cli("ingest", "--root", "ref", "--tag", "reference", "--db", db, cwd=tree)
    assert "ingested 0 new rows" in cli("ingest", "--root", "ours", "--db", db, cwd=tree)  # SHA1 dedup
    src = cli("query", "SELECT source, COUNT(*) n FROM runs GROUP BY source ORDER BY source", "--db", db, cwd=tree)
    assert "reference-log" in src and "reference-harness-csv" in src and "anx-native" in src and "bench" in src
    sp = cli("speedup", "--db", db, cwd=tree)
    row = next(line.split() for line in sp.splitlines() if line.split()[:4] == ["anx-native", "1", "v2.2", "4"])
    assert float(row[5]) == pytest.approx(40.0 / 16.0, abs=1e-3)  # speedup vs v1 np1
    assert float(row[7]) == pytest.approx(40.0 / 16.0 / 4, abs=1e-3)  # self-relative efficiency
    cli("plot", "efficiency", "--out", "e.png", "--source", "anx-native", "--db", db, cwd=tree)
    assert (tree / "e.png").stat().st_size > 1000
    assert "wrote 9 rows" in cli("export", "--fmt", "csv", "--out", "runs.csv", "--db", db, cwd=tree)
    cli("report", "--out", "r.md", "--db", db, "--ref-root", str(tree / "ref"), "--repo-root", ROOT, cwd=tree)
    rep = (tree / "r.md").read_text()
    # ours vs the reference's logged runs: v1 600 / 40 = 15x, v3 200 / 0.2 = 1000x
    assert "| v1        |    1 |    40.000 |             600.000 |                   15.000 |" in rep
    assert "1000.000" in rep
    # Karp-Flatt of v2.2 at np 2: S = 1.6 -> e = (1/1.6 - 1/2) / (1 - 1/2) = 0.25
    kf = next(line for line in rep.splitlines() if "| anx-native" in line and "v2.2" in line and "|    2 |" in line)
    assert kf.rstrip(" |").endswith("0.250")
    assert "Code size per version" in rep
