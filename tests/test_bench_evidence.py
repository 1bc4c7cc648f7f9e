"""bench.py attaches counter evidence only to the code object it was collected
on: profiles/.../pmc_bench_<cfg>.json records the kernel key of
the passes' code object, and a line that timed another one gets traffic null
with the reason.  CPU only: the key comes from the scene's generated source."""
import json
import os

import pytest

import bench


def test_kernel_key_is_the_code_object_key(built):
    from pathtrace import scenes
    cfg = scenes.CONFIGS["C3"]
    k1 = cfg.device_scene().kernel_key(cfg.depth)
    k2 = cfg.device_scene().kernel_key(cfg.depth)
    assert k1 == k2 and len(k1) == 16
    # another depth is another kernel
    assert cfg.device_scene().kernel_key(cfg.depth + 1) != k1
    # the key names the code-object cache entry build() produced for the bench config
    cache = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "path-trace_amd", "_jit_cache")
    if os.path.isdir(cache) and any(f.endswith(".hsaco") for f in os.listdir(cache)):
        assert os.path.exists(os.path.join(cache, k1 + ".hsaco"))


def test_pmc_evidence_bound_to_key(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "PMC_JSON", str(tmp_path / "pmc_bench_%s.json"))
    ev, why = bench.pmc_evidence("C3", "0123456789abcdef")
    assert ev is None and "no counter file" in why
    (tmp_path / "pmc_bench_C3.json").write_text(json.dumps({"kernel_key": "fedcba9876543210",
                                                            "hbm_bytes_per_launch": 1.0}))
    ev, why = bench.pmc_evidence("C3", "0123456789abcdef")
    assert ev is None and "fedcba9876543210" in why and "0123456789abcdef" in why
    ev, why = bench.pmc_evidence("C3", "fedcba9876543210")
    assert why is None and ev["hbm_bytes_per_launch"] == 1.0


@pytest.mark.parametrize("cfg", ["C3", "C2", "C5"])
def test_committed_pmc_files_carry_a_key(cfg):
    path = bench.PMC_JSON % cfg
    if not os.path.exists(path):
        pytest.skip("no committed counter file for %s yet" % cfg)
    with open(path) as f:
        ev = json.load(f)
    assert len(ev.get("kernel_key", "")) == 16
    assert ev["hbm_bytes_per_launch"] > 0 and ev["avg_launch_ms"] > 0
