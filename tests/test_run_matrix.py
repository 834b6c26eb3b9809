"""The staged-version matrix driver (the reference's scripts/0_run_final_project.sh
and scripts/common_test_utils.sh:229-327): CPU-only session at batch 1 — every CPU version and np
must parse, have shape 13x13x256 and the serial checksum, and land in the 20-column CSV."""
import csv
import glob
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_matrix_cpu_only(tmp_path):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run(["bash", os.path.join(ROOT, "scripts", "run_matrix.sh"), "--no-build", "--cpu-only",
                          "--batch", "1", "--iters", "1", "--out", str(tmp_path)],
                         capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    rows = [l.split() for l in out.stdout.splitlines() if l.startswith(("v1 ", "v2.1 ", "v2.2 "))]
    assert [(r[0], r[1]) for r in rows] == [("v1", "1")] + [(v, n) for v in ("v2.1", "v2.2") for n in ("1", "2", "4")]
    assert {r[4] for r in rows} == {"13x13x256"} and {r[5] for r in rows} == {"OK"}
    assert len({r[6] for r in rows}) == 1  # every decomposition == serial V1, bit for bit
    (path,) = glob.glob(str(tmp_path / "matrix_*" / "summary_report_*.csv"))
    with open(path) as f:
        recs = list(csv.reader(f))
    assert len(recs[0]) == 20 and len(recs) == 1 + len(rows)
    assert all(len(r) == 20 for r in recs)
