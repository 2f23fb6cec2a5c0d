"""bench.py's multi-GPU launch contract: with WORLD_SIZE
unset, --gpus N > 1 starts the N ranks itself under torch.distributed.run (a
child process, before the GPU is touched); a launcher's WORLD_SIZE must equal
--gpus.  CPU only: nothing here reaches a GPU call."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_world_size_mismatch_exits_nonzero():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2
    assert "WORLD_SIZE=2 but --gpus 4" in r.stderr


def test_gpus_n_spawns_ranks(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench

    calls = []

    def fake_call(cmd):
        calls.append(cmd)
        return 7

    monkeypatch.setattr(subprocess, "call", fake_call)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "3"])
    try:
        bench.main()
        raise AssertionError("bench.main returned")
    except SystemExit as e:
        assert e.code == 7  # the child's status
    (cmd,) = calls
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == [os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "3"][-4:]
    assert cmd[-5] == os.path.join(ROOT, "bench.py")
