"""bench.py end to end on one GPU (BASELINE metric line).

N = 1: the line carries the timed step's D2H, the one-time costs, the CPU
baseline on the usable host cores with a 1-process rate, and the bit-for-bit
parity of the baseline's pixels. N = 2: two ranks rehearsed on the one GPU
over gloo (RCCL refuses two ranks on one device; the 8-GPU RCCL run is the
driver's) render the strong-scaled frame, and the gathered FP64 frame's
sampled rows match the reference itself (oracle/_ref/ref_render) bit for bit,
rows of both ranks included.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _last_json(out: str) -> dict:
    lines = [l for l in out.splitlines() if l.startswith("{") and '"metric"' in l]
    assert lines, out[-2000:]
    return json.loads(lines[-1])


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _require_ref() -> None:
    """The reference build (oracle/_ref/ref_render, built here and shipped with
    the tree) is the checker of these lines: without it they would check
    nothing, so its absence fails the test instead of passing it."""
    path = os.path.join(ROOT, "oracle", "_ref", "ref_render")
    assert os.path.exists(path), f"{path} missing: build it with `make -C oracle` (needs /root/reference)"


def test_bench_single_gpu_line():
    _require_ref()
    r = subprocess.run([sys.executable, "bench.py", "--config", "c1", "--steps", "3", "--warmup",
                        "1", "--cpu-seconds", "1"], cwd=ROOT, capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 1 and d["scaling"] == "strong" and d["config"]["config_id"] == "c1"
    assert "D2H" in d["timed_step"]
    assert d["one_time_ms"]["set_scene"] >= 0 and d["one_time_ms"]["camera_lists"] >= 0
    assert len(d["per_rank"]) == 1
    # the timed launch's frames: the last against a one-frame render of its seed,
    # the first against the counting kernel's frame of the same seed
    bc = d["batch_check"]
    assert bc["last_frame_equal"] is True and bc["first_frame_equal_counting_kernel"] is True, bc
    assert bc["frames_in_last_timed_launch"] == d["frames_per_launch"] == 3
    cb = d["cpu_baseline"]
    assert cb["kind"] == "reference" and cb["cores"] >= 1 and cb["one_thread_value"] > 0
    assert "cpu_model" in cb and "nproc" in cb
    assert d["parity_vs_cpu"]["fp64_bit_identical"] is True
    # the roofline's executed work, by kind (counting variant)
    rf = d["roofline"]
    assert rf["full_sphere_tests_per_launch"] > 0 and rf["frac"] > 0


def test_bench_frames_in_flight_line():
    """One frame per launch, two launches in flight (each gated on the
    previous one's drain, each reduced by psrt_reduce_lean beside the next
    trace): the timed frames are the reference's, and a batched line's
    `unbatched` rate reports both schedules."""
    _require_ref()
    r = subprocess.run([sys.executable, "bench.py", "--config", "c2", "--steps", "6", "--warmup",
                        "2", "--batch", "1", "--pipeline", "2", "--cpu-seconds", "1"], cwd=ROOT,
                       capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert d["frames_in_flight"] == 2 and d["frames_per_launch"] == 1
    assert d["batch_check"]["last_frame_equal"] is True, d["batch_check"]
    assert d["parity_vs_cpu"]["fp64_bit_identical"] is True
    r = subprocess.run([sys.executable, "bench.py", "--config", "c2", "--steps", "8", "--warmup",
                        "2", "--no-cpu-baseline", "--chain"], cwd=ROOT, capture_output=True, text=True,
                       timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    # batched: one launch of 8, or a chain of 4 / 2 in flight, whichever measured faster
    tm = d["depth_tuning_ms"]
    assert set(tm) == {"b8x1", "b4x2", "b2x2"}, tm
    assert (d["frames_per_launch"], d["frames_in_flight"]) in ((8, 1), (4, 2), (2, 2))
    assert d["batch_check"]["last_frame_equal"] is True, d["batch_check"]
    u = d["unbatched"]
    assert u["frames_in_flight"] in (1, 2) and u["ms_per_step_one_at_a_time"] > 0
    assert u["ms_per_step_two_in_flight"] > 0
    assert u["ms_per_step"] == min(u["ms_per_step_one_at_a_time"], u["ms_per_step_two_in_flight"])


def test_bench_two_ranks_gathered_frame_matches_reference():
    _require_ref()
    env = dict(os.environ, PSRT_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1",
               OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--gpus", "2", "--config", "c1", "--steps", "3", "--warmup", "1", "--pipeline", "1"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["config"]["config_id"] == "c1"
    assert sorted(p["rank"] for p in d["per_rank"]) == [0, 1]
    assert sum(p["rows"] for p in d["per_rank"]) == 225
    par = d["parity_vs_cpu"]
    assert par["checked"] is True, par
    assert par["fp64_bit_identical"] is True and par["ranks_covered"] == 2, par
    # one node: the ranks assemble the frame in shared page-locked host memory
    assert d["frame_to_host"] == "host", d["frame_to_host"]
    assert d["host_frame_check"]["frame_equals_quantized_gathered_fp64"] is True, d["host_frame_check"]


def test_bench_two_ranks_gather_path():
    """--assemble gather: the rows gathered to rank 0 by the collective (RCCL
    on the driver's node; gloo here), then copied to host on rank 0."""
    _require_ref()
    env = dict(os.environ, PSRT_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1",
               OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--gpus", "2", "--config", "c1", "--steps", "3", "--warmup", "1", "--pipeline", "1",
           "--assemble", "gather"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert d["frame_to_host"] == "gather" and "host_frame_check" not in d
    par = d["parity_vs_cpu"]
    assert par["checked"] is True and par["fp64_bit_identical"] is True, par


def test_bench_two_ranks_c4_gathered_frame_checked():
    """The BASELINE's 8-GPU configuration (C4, 3840x2160x500), rehearsed at
    N = 2 over gloo: the gathered timed frame is checked against the
    reference at its full 500 spp on a column window covering both ranks'
    rows, and the timed launch's frames against one-frame renders."""
    _require_ref()
    env = dict(os.environ, PSRT_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1",
               OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--gpus", "2", "--config", "c4", "--steps", "1", "--warmup", "0"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=280, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["config_id"] == "c4"
    assert d["batch_check"]["last_frame_equal"] is True, d["batch_check"]
    assert d["batch_check"]["all_ranks_equal"] is True, d["batch_check"]
    par = d["parity_vs_cpu"]
    assert par["checked"] is True, par
    assert par["fp64_bit_identical"] is True and par["ranks_covered"] == 2, par
    assert par["spp"] == 500, par
    assert d["host_frame_check"]["frame_equals_quantized_gathered_fp64"] is True, d["host_frame_check"]


def test_bench_eight_ranks_driver_command():
    """The driver's 8-GPU command (torchrun --nproc-per-node 8 bench.py --gpus 8),
    rehearsed with 8 ranks on the one GPU over gloo: every
    rank reports, the gathered frame's sampled rows cover all 8 ranks and match
    the reference bit for bit, and every rank's timed launch equals its
    one-frame render. profiles/r06_rehearsal8 holds the C3 and C4 lines."""
    _require_ref()
    env = dict(os.environ, PSRT_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1",
               OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--gpus", "8", "--config", "c1", "--steps", "3", "--warmup", "1"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=200, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 8 and d["scaling"] == "strong" and d["config"]["config_id"] == "c1"
    assert sorted(p["rank"] for p in d["per_rank"]) == list(range(8))
    assert sum(p["rows"] for p in d["per_rank"]) == 225
    par = d["parity_vs_cpu"]
    assert par["checked"] is True and par["fp64_bit_identical"] is True, par
    assert par["ranks_covered"] == 8, par
    bc = d["batch_check"]
    assert bc["all_ranks_equal"] is True and bc["last_frame_equal"] is True, bc
    hc = d["host_frame_check"]
    assert d["frame_to_host"] == "host" and hc["assembled_by"] == 8, hc
    assert hc["frame_equals_quantized_gathered_fp64"] is True, hc
