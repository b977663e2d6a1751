"""bench.py's N > 1 path, run as the driver runs it (torch.distributed.run, one process per rank) with
two and eight ranks on the box's one GPU: each rank renders its row bands with the HIP kernels, the bands are
all-gathered (gloo on host-staged bands: RCCL needs one GPU per rank) and reassembled on rank 0; the
time is the MAX over ranks.  The JSON line must report the whole job (n_gpus 2, both ranks' times, value
from the slowest) and rank 0's reassembled frame must equal the one-rank frame bit for bit (the RNG is
keyed by the global pixel).  The RCCL branch's calls (init_process_group("nccl"), the
all_gather_into_tensor and the MAX all-reduce) run here with one rank (`--force-dist`,
test_bench_rccl_branch_one_rank); their multi-rank data movement runs only on a multi-GPU node (the
driver's scaling run)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from _rt import rt

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H, SPP = 96, 70, 8


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,W,H", [(2, W, H), (8, 64, 1080)])
def test_bench_gloo_matches_one_rank(tmp_path, world, W, H):
    """world 2, and world 8 -- the size the driver's scaling run launches -- on C4's 1080 rows: 135 bands of 8
    rows over 8 ranks, so 7 ranks own 17 bands and one owns 16 (the gather pads the short rank)"""
    img = tmp_path / "frame.npy"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world), "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"), "--gpus", str(world), "--dist-backend", "gloo",
           "--steps", "2", "--warmup", "1", "--width", str(W), "--height", str(H), "--spp", str(SPP), "--no-cpu-baseline",
           "--no-fast-probe", "--dump-image", str(img)]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == world and line["config"]["dist_backend"] == "gloo"
    ranks = line["rank_elapsed_s"]
    assert len(ranks) == world
    # value is the whole job over the slowest rank's time
    assert abs(line["value"] - W * H * SPP * 2 / max(ranks) / 1e6) <= 1e-2 * line["value"]
    assert line["roofline"]["kernel_ms"] > 0
    # where each rank's time went: per rank, the render, the band gather and the closing
    # barrier's wait are disjoint intervals of its timed region
    rt_ms = line["rank_times_ms"]
    for k in ("render_ms", "kernel_ms", "prepass_ms", "gather_ms", "barrier_wait_ms", "render_events_ms", "elapsed_ms"):
        assert len(rt_ms[k]) == world, k
    for i in range(world):
        parts = rt_ms["render_events_ms"][i] + rt_ms["gather_ms"][i] + rt_ms["barrier_wait_ms"][i]
        assert parts <= rt_ms["elapsed_ms"][i] * 1.01 + 1.0, (i, parts, rt_ms["elapsed_ms"][i])
        assert rt_ms["kernel_ms"][i] + rt_ms["prepass_ms"][i] <= rt_ms["render_ms"][i] * 1.01 + 0.5
        assert rt_ms["render_ms"][i] <= rt_ms["render_events_ms"][i] * 1.01 + 0.5
        assert rt_ms["kernel_ms"][i] > 0 and rt_ms["gather_ms"][i] > 0
        assert abs(rt_ms["elapsed_ms"][i] - 1e3 * ranks[i]) <= 0.01 * rt_ms["elapsed_ms"][i] + 0.5
    gathered = np.load(img)
    c = rt.Context(0)
    try:
        c.upload(rt.Scene.cornell())
        c.resize(W, H)
        cam, _, _ = rt.camera_default(W, H)
        one, _ = c.render(cam, SPP, seed=0)
    finally:
        c.close()
    assert np.array_equal(gathered, np.ascontiguousarray(one).view(np.uint32).reshape(H, W))


@pytest.mark.parametrize("W,H,spp", [(W, H, SPP), (1920, 1080, 1024)], ids=["small", "c4"])
def test_bench_rccl_branch_one_rank(tmp_path, W, H, spp):
    """bench.py's RCCL branch executed, not emulated -- torch.distributed.run with ONE rank
    and --force-dist: init_process_group("nccl"), dist.py's all_gather_into_tensor of the RGBA8 bands on
    device tensors, the all_gather of the rank times and the MAX all_reduce, the barriers, and (at the C4
    shape) frame_parity's all_reduces over RCCL.  Not a scaling claim: one rank, one GPU.  The JSON line
    must report the collectives and the gathered frame must equal a plain render bit for bit."""
    img = tmp_path / "frame.npy"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"), "--gpus", "1", "--force-dist", "--dist-backend", "nccl",
           "--steps", "2", "--warmup", "1", "--width", str(W), "--height", str(H), "--spp", str(spp), "--no-cpu-baseline",
           "--no-fast-probe", "--no-c5", "--no-small-configs", "--dump-image", str(img)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=REPO)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and line["config"]["dist_backend"] == "nccl"
    assert line["collectives"]["backend"] == "nccl" and line["collectives"]["forced_one_rank"] is True
    assert len(line["rank_elapsed_s"]) == 1
    assert abs(line["value"] - W * H * spp * 2 / line["rank_elapsed_s"][0] / 1e6) <= 1e-2 * line["value"]
    if spp == 1024:
        assert line["parity"]["sha_match"] is True and line["parity"]["rmse_vs_ref"] == 0.0
    gathered = np.load(img)
    c = rt.Context(0)
    try:
        c.upload(rt.Scene.cornell())
        c.resize(W, H)
        cam, _, _ = rt.camera_default(W, H)
        one, _ = c.render(cam, spp, seed=0)
    finally:
        c.close()
    assert np.array_equal(gathered, np.ascontiguousarray(one).view(np.uint32).reshape(H, W))
