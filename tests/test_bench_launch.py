"""bench.py's self-launch on the CPU: the N-rank child runs in a process group of its
own and is killed as a group past its limit -- a stalled rank cannot hang the command -- and the GPU
count comes from the environment / device nodes, never from HIP. No GPU needed."""
import os
import subprocess
import sys
import time
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def _bench():
    import bench
    return bench


def test_run_group_kills_the_whole_group_on_expiry(tmp_path):
    """A leader that starts a grandchild and then stalls: after the limit the leader AND the grandchild
    are gone, the call returns 124 within limit + grace, and says so on stderr."""
    bench = _bench()
    pidf = tmp_path / "grandchild.pid"
    script = (f"import subprocess, time, sys; p = subprocess.Popen([sys.executable, '-c', 'import time; time.sleep(600)']); "
              f"open({str(pidf)!r}, 'w').write(str(p.pid)); time.sleep(600)")
    t0 = time.monotonic()
    rc = bench.run_group([sys.executable, "-c", script], dict(os.environ), 3.0, "the test ranks", grace=2.0)
    el = time.monotonic() - t0
    assert rc == 124 and el < 3.0 + 2 * 2.0 + 5.0, (rc, el)
    gpid = int(pidf.read_text())
    time.sleep(0.5)
    try:
        os.kill(gpid, 0)
        alive = True
    except ProcessLookupError:
        alive = False
    if alive:  # (a zombie that init has not reaped yet counts as gone)
        st = Path(f"/proc/{gpid}/stat").read_text().split()[2] if Path(f"/proc/{gpid}/stat").exists() else "X"
        alive = st not in ("Z", "X")
    assert not alive, "the stalled rank's child survived the group kill"


def test_run_group_passes_the_exit_code_through():
    bench = _bench()
    assert bench.run_group([sys.executable, "-c", "import sys; sys.exit(3)"], dict(os.environ), 30.0, "x") == 3
    assert bench.run_group([sys.executable, "-c", "pass"], dict(os.environ), 30.0, "x") == 0


def test_visible_gpus_from_the_environment(monkeypatch):
    bench = _bench()
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,3,5")
    assert bench.visible_gpus() == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert bench.visible_gpus() == 0


def test_gpus2_without_enough_gpus_fails_fast_with_a_message():
    """Two ranks asked for, none visible (this container): a message and exit 2, before anything
    starts -- and this parent never imports HIP state (it would have to initialise it to count)."""
    env = dict(os.environ, HIP_VISIBLE_DEVICES="")
    env.pop("RSORT_BENCH_BACKEND", None)
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2"], capture_output=True, text=True,
                       timeout=300, env=env, cwd=str(ROOT))
    assert r.returncode == 2 and "GPU(s) visible" in r.stderr, (r.returncode, r.stderr[-1000:])


def test_launch_timeout_default_scales_with_the_job():
    bench = _bench()

    class A:
        launch_timeout = 0.0
        n = 1 << 30
        gpus = 8
    assert bench.launch_timeout(A) == 300.0 + 60.0 * 8
    A.launch_timeout = 42.0
    assert bench.launch_timeout(A) == 42.0


def test_comm_timeout_setting_needs_no_device():
    sys.path.insert(0, str(ROOT / "cuda.radixsort_amd"))
    import radixsort as rs
    old = rs.set_comm_timeout(4321)
    try:
        assert rs.set_comm_timeout(-1) == 4321  # (<= 0 leaves it unchanged)
        assert rs.set_comm_timeout(0) == 4321
    finally:
        rs.set_comm_timeout(old)
    with pytest.raises(rs.RSortError) as e:
        rs.RcclComm(2, 5, bytes(128))  # rank outside the world: refused before RCCL is touched
    assert e.value.status == 1
