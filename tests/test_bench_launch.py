"""bench.py's multi-GPU launch (CPU): `python3 bench.py --gpus N` starts N rank processes
itself when no launcher set WORLD_SIZE (the reference's join_init_run spawns its own
worker threads, radix_join.cpp:1531-1540), relays rank 0's line, and exits with the
worst rank's status; without N GPUs (RCCL backend) it refuses, and it never prints a
line for a different number of GPUs than asked."""
import json
import os
import subprocess
import sys
import time

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402

RANK_SCRIPT = r"""
import json, os, sys, time
r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
print(json.dumps({"rank": r, "world": w, "local": int(os.environ["LOCAL_RANK"]),
                  "addr": os.environ["MASTER_ADDR"], "port": int(os.environ["MASTER_PORT"])}), flush=True)
if os.environ.get("HANG_RANK") == str(r):
    time.sleep(600)
sys.exit(int(os.environ.get("FAIL_CODE", "0")) if os.environ.get("FAIL_RANK") == str(r) else 0)
"""


def _run(capsys, n, grace_s=60.0, **env):
    rc = bench.launch_ranks([sys.executable, "-c", RANK_SCRIPT], n, grace_s=grace_s, env_extra=env)
    out = capsys.readouterr()
    return rc, [ln for ln in out.out.splitlines() if ln.strip()], out.err


def test_launch_relays_rank0_only(capsys):
    rc, lines, err = _run(capsys, 4)
    assert rc == 0
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["rank"] == 0 and d["world"] == 4 and d["local"] == 0 and d["addr"] == "127.0.0.1" and d["port"] > 0
    for r in (1, 2, 3):  # the other ranks' stdout goes to stderr
        assert f"[rank {r} stdout]" in err


def test_launch_worst_status(capsys):
    rc, lines, _ = _run(capsys, 3, FAIL_RANK="2", FAIL_CODE="3")
    assert rc == 3 and len(lines) == 1


def test_launch_terminates_hung_peers(capsys):
    """Rank 1 fails while rank 2 hangs (as in a collective the failed rank never
    reaches): after the grace period rank 2 is terminated; the status reports it."""
    t0 = time.monotonic()
    rc, lines, err = _run(capsys, 3, grace_s=1.0, FAIL_RANK="1", FAIL_CODE="5", HANG_RANK="2")
    assert time.monotonic() - t0 < 60
    assert rc == 128 + 15  # SIGTERM outranks the failed rank's 5
    assert "a rank failed" in err


def test_bench_refuses_without_gpus():
    """No GPU here: --gpus 2 over RCCL cannot get a GPU per rank -> non-zero, no line."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                         text=True, timeout=300, env={k: v for k, v in os.environ.items() if k != "WORLD_SIZE"})
    assert out.returncode == 2
    assert out.stdout.strip() == ""
    assert "needs 2 visible GPUs" in out.stderr


def test_bench_refuses_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                         text=True, timeout=300, env=env)
    assert out.returncode == 2 and out.stdout.strip() == ""
    assert "refusing to measure" in out.stderr


@pytest.mark.parametrize("kernel,expect", [("R_pass1_scatter", 13), ("S_pass2_scatter", 8), ("join_build_probe", 4)])
def test_algorithmic_bytes_keys_layout(kernel, expect):
    """Bytes per tuple the roofline prices (keys layout, 7-bit pass-2 digit)."""
    n = 1 << 20
    per = bench.algorithmic_bytes(kernel, n, n, 2, 7, 4) / (n * (2 if kernel == "join_build_probe" else 1))
    assert per == expect


@pytest.mark.parametrize("kernel,narrow,expect", [("R_pass2_scatter", 3, 6), ("S_pass2_scatter", 1, 8),
                                                  ("S_pass2_scatter", 2, 6), ("R_pass1_scatter", 3, 13),
                                                  ("join_build_probe", 3, 2), ("join_build_probe", 1, 3)])
def test_algorithmic_bytes_narrow(kernel, narrow, expect):
    """Narrow partitions (stats narrow bit 0 R / bit 1 S): pass 2 writes and the build/probe
    reads 2-byte residuals; pass 1 is unchanged."""
    n = 1 << 20
    per = bench.algorithmic_bytes(kernel, n, n, 2, 7, 4, 2, narrow) / (n * (2 if kernel == "join_build_probe" else 1))
    assert per == expect
