"""bench.py's own multi-rank launcher (`python bench.py --gpus N` without torchrun) must fail
loudly: a rank killed by a signal makes the launcher exit non-zero, and its siblings are
stopped instead of being left blocked in a collective (the driver's 8-GPU scaling run goes
through this code; the reference's exchange is communication.py:246-291)."""
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_rank_exit_code_maps_signals():
    assert bench.rank_exit_code(0) == 0
    assert bench.rank_exit_code(3) == 3
    assert bench.rank_exit_code(-6) == 134   # SIGABRT, as a shell reports it
    assert bench.rank_exit_code(-11) == 139  # SIGSEGV


def test_wait_ranks_signal_stops_siblings():
    """One child aborts, the other would sleep for a minute: the launcher returns 134 at
    once and the sleeper is gone."""
    abort = subprocess.Popen([sys.executable, "-c", "import os, signal, time; time.sleep(0.5); "
                                                    "os.kill(os.getpid(), signal.SIGABRT)"])
    sleeper = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(60)"])
    t0 = time.time()
    rc = bench.wait_ranks([sleeper, abort])
    assert rc == 134
    assert time.time() - t0 < 20
    assert sleeper.poll() is not None


def test_wait_ranks_all_ok():
    ps = [subprocess.Popen([sys.executable, "-c", "pass"]) for _ in range(3)]
    assert bench.wait_ranks(ps) == 0


def test_wait_ranks_nonzero_exit():
    ok = subprocess.Popen([sys.executable, "-c", "pass"])
    bad = subprocess.Popen([sys.executable, "-c", "import sys; sys.exit(7)"])
    assert bench.wait_ranks([ok, bad]) == 7


@pytest.mark.timeout(120)
def test_bench_gloo_world2_rank_abort_fails_launcher():
    """The real launcher path: `bench.py --gpus 2 --backend gloo`, rank 1 aborts (SIGABRT)
    right after init_process_group, rank 0 blocks in the first collective.  The launcher must
    exit non-zero well before the collective's own timeout."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--die-before-exchange", "1", "--dist-timeout", "90"],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode != 0, r.stderr[-2000:]
    assert r.returncode in (1, 134), (r.returncode, r.stderr[-2000:])
    assert time.time() - t0 < 80
