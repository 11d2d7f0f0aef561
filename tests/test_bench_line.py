"""GPU: the default bench line (what the driver records each round) carries the headline plus the
other BASELINE configs -- config 5 (bunny-class proxy), config 2 (1080p, 2 bounces) and config 3 in
the CPU-parity math -- each with its own timing and roofline, and the headline's roofline prices
the overlapped accumulation beside the render (bench.py, EXTRA_CONFIGS)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_default_bench_line_carries_every_config():
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline", "--no-drop-in"], capture_output=True, text=True, timeout=240, cwd=REPO)
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["value"] > 0
    assert set(line["roofline"]) >= {"accum_valu_insts_per_launch", "frac_with_accum", "lane_util"}
    cfg = line["configs"]
    assert set(cfg) == {"cfg5_bunny", "cfg2_1080p", "cfg3_pinned"}
    for name, c in cfg.items():
        assert c["ms_per_frame"] > 0 and c["value"] > 0 and c["rays_per_step"] > 0, name
        assert c["roofline"]["bound"] == "valu" and c["roofline"]["launch_ms"] > 0, name
    assert cfg["cfg5_bunny"]["workload"].startswith("bunny 3840x2160 8spp 9-bounce")
    assert cfg["cfg2_1080p"]["workload"] == "cornell 1920x1080 1spp 2-bounce path trace"
    assert cfg["cfg3_pinned"]["math"] == "pinned"
    # pinned and shipped render the same paths: Intersect() counts differ only where the maths
    # flip a hit (SURVEY.md 7 hard part 1), by far less than a percent
    rel = abs(cfg["cfg3_pinned"]["rays_per_step"] - line["config"]["rays_per_step"]) / line["config"]["rays_per_step"]
    assert rel < 1e-3


def test_every_bench_config_has_a_pmc_record():
    """CPU: the headline and every extra config of the default bench line are priced by a
    profiles/pmc.json record (scripts/profile.sh); `stale` in the line says whether the record was
    measured on the current kernel sources."""
    import bench
    db = json.load(open(os.path.join(REPO, "profiles", "pmc.json")))
    base = bench.parse([])
    keys = [bench.workload_key(base, 1, base.frames)]
    for _, over, _, _ in bench.EXTRA_CONFIGS:
        a = bench.parse([])
        a.__dict__.update(over)
        keys.append(bench.workload_key(a, 1, a.frames if a.frames > 1 else 1))
    missing = [k for k in keys if k not in db]
    assert not missing, f"no PMC record for {missing} (run scripts/profile.sh)"
    assert len(set(keys)) == len(keys)
