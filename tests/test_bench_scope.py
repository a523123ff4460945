"""bench.py's roofline record (CPU): t_probe always holds every S partition
pass; the distributed path's local-only figure is reported
under its own name; the copy floor prices the phase's structural bytes at the
box's own copy rates."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

GB = 12_884_901_888      # C3: 48 B x 2^28
READ = 8_589_934_592
FLOOR = {"persistent_gbs": 5500.0, "flat_gbs": 6300.0}


def test_single_gpu_scope_is_t_probe():
    r = bench.probe_roofline("radix", False, 5.0, 0.0, GB, READ)
    assert r["scope"] == bench.SCOPE_T_PROBE
    assert r["ms"] == 5.0
    assert r["frac"] == pytest.approx(GB / 5e-3 / 1e9 / 8000.0, abs=1e-4)
    assert "local_probe" not in r


def test_distributed_frac_includes_s_routing():
    r = bench.probe_roofline("radix", True, 4.2, 2.2, GB, READ)
    # the t_probe figure carries S's route (its first partition pass)
    assert r["scope"] == bench.SCOPE_T_PROBE_DIST
    assert r["ms"] == pytest.approx(6.4)
    assert r["frac"] == pytest.approx(GB / 6.4e-3 / 1e9 / 8000.0, abs=1e-4)
    assert r["s_route_ms"] == 2.2
    # the local-only figure is labelled as NOT t_probe
    lp = r["local_probe"]
    assert lp["ms"] == 4.2 and lp["frac"] > r["frac"]
    assert "NOT t_probe" in lp["scope"]


@pytest.mark.parametrize("use_dist,route", [(False, 0.0), (True, 0.0), (True, 1.7)])
def test_no_t_probe_scope_excludes_an_s_pass(use_dist, route):
    """Whatever the path, a record whose scope names t_probe times S's route
    when there is one (a replicated R has none: S keeps all its passes)."""
    r = bench.probe_roofline("radix", use_dist, 4.0, route, GB, READ)
    assert "t_probe" in r["scope"] and "NOT t_probe" not in r["scope"]
    assert r["ms"] == pytest.approx(4.0 + route)
    for k, v in r.items():
        if isinstance(v, dict) and "scope" in v and "t_probe" in v["scope"]:
            assert "NOT t_probe" in v["scope"], k


def test_copy_floor_fields():
    struct = 30_064_771_072   # C3: 2 S passes x 32 B + the join's 48 B, x 2^28
    r = bench.probe_roofline("radix", False, 5.96, 0.0, GB, READ, structure_bytes=struct, floor=FLOOR)
    assert r["floor_ms"] == pytest.approx(struct / 5500e6, abs=1e-3)
    assert r["floor_flat_ms"] == pytest.approx(struct / 6300e6, abs=1e-3)
    assert r["phase_over_floor"] == pytest.approx(5.96 / (struct / 5500e6), abs=1e-3)
    # no floor for the global-table strategy (not a streamed structure)
    g = bench.probe_roofline("global", False, 9.0, 0.0, GB, READ, structure_bytes=struct, floor=FLOOR)
    assert g["scope"] == bench.SCOPE_GLOBAL and "floor_ms" not in g
