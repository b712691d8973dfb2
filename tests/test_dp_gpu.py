"""The multi-rank step with the real HIP kernels (-m gpu), rehearsed on one GPU.

``bench.py --gpus 2 --backend gloo --config C4`` starts two ranks (fresh child processes, one GPU
shared), each rendering its round-robin half of the 27-camera rig with the deferred multi-view
backward accumulating into the flat gradient bucket, then one SUM all-reduce of the bucket
(splat_dp.GradAllReduce, the 56 MB C4 bucket).  ``--grad-checksum`` saves both ranks' reduced bucket
of one further step.  It must equal a single-process backward of the same 27 views summed
(train.py:413-418 sums the view losses) within 1e-5 relative (+ 1e-6 x max per array:
the per-rank partial sums group the fp32 additions differently), and both ranks must hold the same
bucket.  (RCCL over xGMI and the 8-GPU run stay with the driver.)
"""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import splat_scenes as S
import splat_step

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_rank_c4_step_equals_single_process(cuda, tmp_path):
    path = str(tmp_path / "c4_bucket")
    cmd = [sys.executable, "-u", os.path.join(REPO, "bench.py"), "--gpus", "2", "--backend", "gloo",
           "--config", "C4", "--steps", "2", "--warmup", "1", "--probe-steps", "0", "--no-cpu-baseline",
           "--grad-checksum", path]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    b = [torch.load(f"{path}.rank{k}.pt", weights_only=True) for k in range(2)]
    assert b[0]["world"] == 2 and b[1]["world"] == 2
    assert sorted(b[0]["views"] + b[1]["views"]) == list(range(27))
    assert torch.equal(b[0]["bucket"], b[1]["bucket"]), "the ranks hold different reduced gradients"
    _equals_single_process_c4(cuda, b[0])


def test_rccl_one_rank_c4_step(cuda, tmp_path):
    """The RCCL code path itself on one GPU: `torch.distributed.run --nproc-per-node 1 bench.py --backend
    nccl` forms a one-rank NCCL (= RCCL) process group (init_process_group("nccl", device_id=...)), the
    flat gradient bucket is all-reduced in place over RCCL every step with the gsr_grad_fence ordering
    the next step's gradient writes behind it, and the reduced bucket of the checksum step equals the
    single-process sum of the 27 rig views."""
    import json
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    path = str(tmp_path / "c4_rccl")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(REPO, "bench.py"), "--gpus", "1",
           "--backend", "nccl", "--config", "C4", "--steps", "2", "--warmup", "1", "--probe-steps", "0",
           "--no-cpu-baseline", "--grad-checksum", path]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["config"]["backend"] == "nccl", line["config"]
    b = torch.load(f"{path}.rank0.pt", weights_only=True)
    assert b["world"] == 1 and sorted(b["views"]) == list(range(27))
    _equals_single_process_c4(cuda, b)


def _equals_single_process_c4(cuda, b):
    """The reduced bucket `b` against one process rendering all 27 C4 views summed."""
    # single process: the same leaves (bench.py's C4 setup), all 27 views summed, one backward
    cfg = S.CONFIGS["C4"]
    p = S.synthetic_cloud(cfg.P, cfg.s0, sh_degree=-1, seed=0, device=cuda)
    with torch.no_grad():
        act = S.activated_inputs(p, -1)
    leaves = {k: v.detach().clone().requires_grad_(True) for k, v in act.items()}
    cams = S.scene_cameras(cfg, device=cuda)
    streams = [torch.cuda.Stream() for _ in range(3)]
    for s in streams:
        s.wait_stream(torch.cuda.current_stream())
    step = splat_step.RenderStep(cuda, cams, lambda ci: leaves, S.upstream_grad(cfg.height, cfg.width, device=cuda),
                                 streams, threads=True)
    try:
        step(list(range(27)))
    finally:
        step.close()
    torch.cuda.synchronize()
    names = b["names"]
    assert names == [k for k in leaves if k != "means2D"]
    got = b["bucket"].numpy().astype(np.float64)
    o = 0
    for k in names:
        ref = leaves[k].grad.detach().cpu().numpy().reshape(-1).astype(np.float64)
        g = got[o:o + ref.size]
        o += ref.size
        err = np.abs(g - ref)
        bad = err > 1e-5 * np.abs(ref) + 1e-6 * np.abs(ref).max()
        assert not bad.any(), f"{k}: {bad.sum()} of {ref.size} off, worst {err.max():.3g} (max |ref| {np.abs(ref).max():.3g})"
    assert o == got.size
