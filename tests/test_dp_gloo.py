"""Multi-process (world_size 2, gloo, CPU) tests of the camera data-parallel path (splat_dp)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import splat_dp

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "reference_harness.npz"))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = {}
        # 1) gradient all-reduce == sum over ranks
        g = torch.Generator().manual_seed(100 + rank)
        params = [torch.nn.Parameter(torch.zeros(7, 3)), torch.nn.Parameter(torch.zeros(5, 4))]
        for p in params:
            p.grad = torch.randn(p.shape, generator=g)
        local = [p.grad.clone() for p in params]
        splat_dp.GradAllReduce(params)()
        out["grads"] = [p.grad.numpy() for p in params]
        out["local"] = [x.numpy() for x in local]
        # 1b) in-place bucket: backward accumulates into the attached bucket, reduce sums over ranks
        ps = [torch.nn.Parameter(torch.ones(7, 3)), torch.nn.Parameter(torch.ones(5, 4))]
        red = splat_dp.GradAllReduce(ps).attach()
        ws = [torch.randn(p.shape, generator=g) for p in ps]
        for _ in range(2):  # two views accumulate
            sum((p * w).sum() for p, w in zip(ps, ws)).backward()
        red.reduce()
        out["inplace"] = [p.grad.clone().numpy() for p in ps]
        out["inplace_local"] = [(2 * w).numpy() for w in ws]
        assert all(p.grad.data_ptr() >= red.flat.data_ptr() for p in ps)  # still views of the bucket
        red.zero_()
        out["inplace_zeroed"] = float(sum(p.grad.abs().sum() for p in ps))
        # 2) densify statistics: views sharded round-robin, then SUM/SUM/MAX
        radii, grads = GOLD["dstat_in_radii"], GOLD["dstat_in_grad"]
        st = splat_dp.DensifyStats(radii.shape[1], "cpu")
        for v in splat_dp.shard_views(list(range(len(radii))), rank, world):
            st.update(torch.from_numpy(radii[v]), torch.from_numpy(grads[v]))
        st.allreduce()
        out["vis"] = st.visibility_count.numpy()
        out["acc"] = st.mean_2d_gradients_accumulated.numpy()
        out["maxr"] = st.max_2d_radii.numpy()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_dp_allreduce_and_densify_stats_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        for a, b0, b1 in zip(res[r]["grads"], res[0]["local"], res[1]["local"]):
            np.testing.assert_allclose(a, b0 + b1, rtol=1e-6, atol=1e-6)
        for a, b0, b1 in zip(res[r]["inplace"], res[0]["inplace_local"], res[1]["inplace_local"]):
            np.testing.assert_allclose(a, b0 + b1, rtol=1e-6, atol=1e-6)
        assert res[r]["inplace_zeroed"] == 0.0
        # sharded accumulation + all-reduce == the reference's sequential accumulation
        np.testing.assert_array_equal(res[r]["vis"], GOLD["dstat_out_visibility_count"])
        np.testing.assert_array_equal(res[r]["maxr"], GOLD["dstat_out_max_radii"])
        np.testing.assert_allclose(res[r]["acc"], GOLD["dstat_out_grad_accum"], rtol=1e-6, atol=1e-9)


def _densify_worker(rank, world, port, q, broadcast):
    """Camera-DP densification on each rank: sharded view statistics -> splat_dp.densify_gaussians with
    the numpy densify oracle as the engine (no GPU here).  Every rank seeds torch differently, so only
    the broadcast draw keeps the split copies identical."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import densify_oracle as DO
        torch.manual_seed(1000 + rank)
        pre = "dens0_pre_"
        keys = [k[len(pre):] for k in GOLD.files if k.startswith(pre) and not k.startswith(pre + "m_")
                and not k.startswith(pre + "v_")]
        params = {k: GOLD[pre + k] for k in keys}
        m = {k: GOLD[pre + "m_" + k] for k in keys if k not in DO.GAUSSIAN_EXCLUDED}
        v = {k: GOLD[pre + "v_" + k] for k in keys if k not in DO.GAUSSIAN_EXCLUDED}
        P = params["means"].shape[0]
        rng = np.random.default_rng(7)  # the same 6 views on every rank; each renders its shard
        radii = rng.integers(0, 5, (6, P)).astype(np.int32)
        grads = (6e-4 * rng.standard_normal((6, P, 3))).astype(np.float32)
        st = splat_dp.DensifyStats(P, "cpu")
        for view in splat_dp.shard_views(list(range(6)), rank, world):
            st.update(torch.from_numpy(radii[view]), torch.from_numpy(grads[view]))

        def engine(params, stats, scene_radius, optimizer, i, sample_fn):
            draw = sample_fn if broadcast else (lambda mean, std: torch.normal(mean=mean, std=std))
            z = np.zeros(P, np.float32)
            return DO.densify(params, m, v, stats.mean_2d_gradients_accumulated.numpy(),
                              stats.visibility_count.numpy(), stats.max_2d_radii.numpy(), z.astype(bool),
                              np.zeros((P, 3), np.float32), scene_radius, i,
                              lambda stds: draw(torch.zeros(stds.shape), torch.from_numpy(stds)).numpy())

        p2, m2, v2, *_rest, info = splat_dp.densify_gaussians(
            params, st, float(GOLD["dens0_scene_radius"]), None, 500, densify_fn=engine)
        q.put((rank, {"p": p2, "m": m2, "v": v2, "n_split": info["n_split"]}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("broadcast", [True, False])
def test_dp_densify_identical_on_all_ranks_world2(broadcast):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_densify_worker, args=(r, world, port, q, broadcast)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0]["n_split"] > 0
    same = all(np.array_equal(res[0][part][k], res[1][part][k]) for part in ("p", "m", "v") for k in res[0][part])
    # the broadcast draw keeps the replicas identical; independent draws make them diverge
    assert same == broadcast


def _bench_dry_run(world, config):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(world), "--dry-run",
                        "--config", config, "--steps", "2"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # exactly one JSON line, from rank 0
    return json.loads(lines[0])


@pytest.mark.parametrize("world,config,shards", [(2, "C4", [14, 13]), (2, "C3", [5, 5]),
                                                 (8, "C4", [4, 4, 4, 3, 3, 3, 3, 3])])
def test_bench_self_launch_dry_run(world, config, shards):
    """bench.py --gpus N with no launcher environment starts N ranks itself (torch.distributed.run
    children, gloo in the dry run), rank 0 prints one JSON line with n_gpus = the process group's
    world size; C4 shards the 27-camera rig round-robin and the per-step all-reduce sums every rank."""
    out = _bench_dry_run(world, config)
    assert out["n_gpus"] == world
    assert out["config"]["views_per_rank"] == shards
    assert out["bucket_sum_ok"]


def test_sharding_partitions():
    views = list(range(27))
    shards = [splat_dp.shard_views(views, r, 8) for r in range(8)]
    assert sorted(sum(shards, [])) == views
    assert [len(s) for s in shards] == [4, 4, 4, 3, 3, 3, 3, 3]
    frames = [splat_dp.shard_frames(150, r, 8) for r in range(8)]
    assert sum((list(f) for f in frames), []) == list(range(150))
    assert [len(f) for f in frames] == [19, 19, 19, 19, 19, 19, 18, 18]
