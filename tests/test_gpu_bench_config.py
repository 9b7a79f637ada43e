"""bench.py's multi-GPU configuration exercised on one GPU: the first 8-GPU run
executes exactly this -- an RCCL-sharded context (prt_shard_init_rccl inside the boundary, one ncclGather per
frame), bench.py's frames in flight on several GPUs with cut chain grids, the process's hardware-queue
setting read before any HIP call -- so it runs here in a child process with those settings, and every frame must
equal the unsharded one bit for bit.  A communicator whose peers never arrive must fail within the time limit
(prt_shard_init_rccl with a non-blocking, polled RCCL set-up) instead of hanging."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _child(args, env_extra, timeout):
    env = dict(os.environ)
    env.update(env_extra)
    r = subprocess.run([sys.executable, os.path.join(HERE, "shard_child.py"), *args], env=env, capture_output=True,
                       text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def _bench_flights():
    """the frames in flight bench.py keeps on several GPUs (its --inflight default for --gpus >= 2)"""
    sys.path.insert(0, os.path.dirname(HERE))
    import bench
    return bench.default_inflight(8)


@pytest.mark.parametrize("queues", ["default", "8"])
def test_bench_multi_gpu_configuration(queues):
    env = {} if queues == "default" else {"GPU_MAX_HW_QUEUES": queues}
    out = _child(["bench", str(_bench_flights()), "960", "540"], env, 240)
    assert out["world"] == 1 and out["frames"] == 6
    assert out["mismatch"] == [] and out["totals_equal"], out


def test_rccl_init_with_missing_peer_fails_in_bounded_time():
    out = _child(["stall"], {"PRT_RCCL_TIMEOUT_S": "4"}, 120)
    assert out["error"] and "did not join" in out["error"], out
    assert out["seconds"] < 30, out
