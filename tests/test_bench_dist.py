"""Multi-process plumbing of bench.py on CPU (gloo, world_size 2): frame sharding and the
max-over-ranks timing reduction used with RCCL on the GPU box."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r, lr, w = bench.dist_env()
    elapsed = 1.0 + rank  # rank 1 is the slow one
    m = bench.dist_max(elapsed, w)
    seeds = [None] * w
    dist.all_gather_object(seeds, bench.shard_seed(0x1080, r))
    q.put((r, lr, w, m, seeds))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_max_and_sharding():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for r, (rank, lr, w, m, seeds) in enumerate(res):
        assert (rank, lr, w) == (r, r, 2)
        assert m == 2.0                       # max over ranks
        assert len(set(seeds)) == 2           # disjoint frame shards


def test_aggregate_is_whole_job_throughput():
    v, ms = bench.aggregate(frames_per_step=8, steps=10, world=4, max_elapsed_s=2.0)
    assert v == 8 * 10 * 4 / 2.0 and ms == 200.0
    assert bench.algorithmic_bytes_per_frame(1920, 1080) == 1920 * 1080 * 2 + 135 * 97840 * 4


def test_gpus_flag_without_launcher_starts_ranks():
    """`bench.py --gpus 2` with no launcher starts two ranks itself (gloo plumbing check on
    CPU): world size 2 in the line, value = all ranks' frames / the slowest rank's time."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, bench.__file__, "--gpus", "2", "--plumbing-check", "--steps", "5",
                        "--frames-per-step", "4"], capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["ranks"]["world_size"] == 2 and line["ranks"]["backend"] == "gloo"
    per = line["ranks"]["per_rank_frames_per_s"]
    assert len(per) == 2 and per[0] > per[1]          # rank 1 sleeps twice as long
    # whole-job rate: 2 ranks x 5 steps x 4 frames over the slowest rank's time (between the
    # barriers), so at most twice the slow rank's own rate
    assert abs(line["value"] - 2 * 5 * 4 / (5 * line["ms_per_step"] * 1e-3)) / line["value"] < 1e-3
    assert line["value"] <= 2 * per[1] * 1.001
    # the end-to-end legs at N > 1: every rank runs them, aggregate = all ranks' frames over the
    # slowest rank's time per round (rank 1 sleeps 20 ms / 10 ms per round), each rank's own rate
    e2e = line["end_to_end"]
    assert e2e["world_size"] == 2 and e2e["frames_per_call"] == bench.E2E_FRAMES_MULTI
    frames = 2 * bench.E2E_CALLS * bench.E2E_FRAMES_MULTI
    for leg, slow_s in (("value", 0.02), ("decisions_value", 0.01)):
        assert 0.5 * frames / slow_s < e2e["aggregate"][leg] <= frames / slow_s, (leg, e2e)
        own = e2e["ranks"][leg]
        assert len(own) == 2 and own[0] > own[1], (leg, own)
        assert len(e2e["rounds"][leg]) == bench.E2E_ROUNDS


def test_gpus_flag_must_match_launcher():
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, bench.__file__, "--gpus", "4", "--plumbing-check"], capture_output=True,
                       text=True, timeout=120, env=env)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


def test_work_knobs_are_refused():
    """A headline number is never measured with a work-changing library knob set
    (MIPGPU_NO_PAIRS searches no mode pair, MIPGPU_SHAPE_FILTER drops shapes, ...): exit 3
    before anything runs; --allow-knobs (A/B tools) lets the run go on and records them."""
    import json
    import subprocess
    import sys
    base = {k: v for k, v in os.environ.items() if not k.startswith("MIPGPU_")
            and k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    for knob in ("MIPGPU_NO_PAIRS", "MIPGPU_SHAPE_FILTER", "MIPGPU_GROUPS", "MIPGPU_LIB"):
        r = subprocess.run([sys.executable, bench.__file__, "--plumbing-check", "--steps", "1"], capture_output=True,
                           text=True, timeout=120, env=dict(base, **{knob: "1"}))
        assert r.returncode == 3 and knob in r.stderr, (knob, r.returncode, r.stderr)
    r = subprocess.run([sys.executable, bench.__file__, "--plumbing-check", "--steps", "1", "--allow-knobs"],
                       capture_output=True, text=True, timeout=120, env=dict(base, MIPGPU_NO_PAIRS="1"))
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip().splitlines()[-1])["n_gpus"] == 1
    # print-only diagnostics do not count
    r = subprocess.run([sys.executable, bench.__file__, "--plumbing-check", "--steps", "1"], capture_output=True,
                       text=True, timeout=120, env=dict(base, MIPGPU_STAGE_STATS="1"))
    assert r.returncode == 0, r.stderr


def test_pmc_profile_of_another_build_is_not_used(tmp_path, monkeypatch):
    """bench.load_pmc takes profiles/traffic.json's numbers only when the entry's build ID
    names the same sources and flags as the loaded library."""
    import json
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "traffic.json").write_text(json.dumps({"64x64x2": {"build_id": "src:aaaa git:x", "hbm_bytes_per_launch": 5}}))
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    rec, why = bench.load_pmc(64, 64, 2, "src:aaaa git:y")
    assert rec["hbm_bytes_per_launch"] == 5 and "same build" in why
    rec, why = bench.load_pmc(64, 64, 2, "src:bbbb git:x")
    assert rec == {} and "src:aaaa" in why
    rec, why = bench.load_pmc(64, 64, 3, "src:aaaa git:x")
    assert rec == {}


def test_valu_section_reports_both_issue_peaks():
    """The `valu` object prices the measured VALU rate against the single-issue rate (`frac`)
    and the two-per-quad-cycle dual-issue peak (`frac_of_dual_peak`)."""
    pmc = {"valu_insts_per_launch": 30.0e9, "valu_issue_utilization": 0.98,
           "valu_insts_per_simd_quad_cycle": 0.98, "valu_dual_issue_share": 0.054}
    v = bench.valu_section(pmc, 50.0, 99.6e6 * 510 * 384)
    rate = 30.0e9 / 0.050
    assert v["frac"] == round(rate / bench.VALU_PEAK_INSTS, 4)
    assert v["frac_of_dual_peak"] == round(rate / (2 * bench.VALU_PEAK_INSTS), 4)
    assert v["dual_peak"] == round(2 * bench.VALU_PEAK_INSTS / 1e9, 1)
    # without a PMC profile of this build the measured fields stay null
    v0 = bench.valu_section({}, 50.0, 1.0)
    assert v0["frac"] is None and "frac_of_dual_peak" not in v0


@pytest.mark.parametrize("world,local_rank", [(8, 5), (8, 0), (2, 1)])
def test_nccl_branch_with_one_device_per_rank(monkeypatch, world, local_rank):
    """The driver's N-GPU run (one rank per GPU, device_count() == WORLD_SIZE): the rank's
    process group is nccl (RCCL) bound to device LOCAL_RANK, and its collectives use that
    device -- checked with the process-group constructor mocked (no GPU here)."""
    calls = []
    monkeypatch.setattr(dist, "init_process_group", lambda *a, **k: calls.append((a, k)))
    backend, dev, coll = bench.init_ranks(world, local_rank, world)
    assert (backend, dev) == ("nccl", local_rank)
    assert coll == torch.device("cuda", local_rank)
    assert calls == [(("nccl",), {"device_id": torch.device("cuda", local_rank)})]


def test_gloo_branch_when_ranks_share_devices(monkeypatch):
    """More ranks than GPUs (the one-GPU rehearsal of the 8-rank run): gloo, rank r on device
    r % count, host-side collectives."""
    calls = []
    monkeypatch.setattr(dist, "init_process_group", lambda *a, **k: calls.append((a, k)))
    assert bench.init_ranks(8, 5, 1) == ("gloo", 0, None)
    assert calls == [(("gloo",), {})]
    calls.clear()
    assert bench.init_ranks(1, 0, 1)[:2] == ("nccl", 0) and calls == []  # one rank: no process group


def test_metric_names_the_frame_size():
    assert bench.metric_name(1920, 1080) == bench.METRIC
    assert bench.metric_name(3840, 2160).startswith("3840x2160 frames/sec")
    assert "1080p" not in bench.metric_name(7680, 4320)
