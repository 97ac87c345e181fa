"""CPU: bench.py's roofline model.  Every per-launch figure must be a ratio of sums over
the same timed launches, so the reported fraction cannot depend on how many steps were timed, and
only the rays the trace launches traversed (not the culled camera rays) are charged."""
import importlib.util
import os
from types import SimpleNamespace

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _step_stats(steps, launches_per_step=6, ms_per_launch=0.3, tp=10_000_000, tb=28_000_000, shadow=12_000_000):
    """The summed stats of `steps` identical timed steps."""
    return SimpleNamespace(trace_launches=launches_per_step * steps, ms_trace=ms_per_launch * launches_per_step * steps,
                           traced_primary=tp * steps, traced_bounce=tb * steps, rays_shadow=shadow * steps,
                           shadow_launches=6 * steps, ms_shadow=0.8 * 6 * steps)


CNT = SimpleNamespace(traced_primary=10_000_000, traced_bounce=28_000_000, node_visits=90_000_000,
                      tri_tests=40_000_000, sphere_tests=5_000_000, node_visits_primary=30_000_000,
                      tri_tests_primary=12_000_000, sphere_tests_primary=1_000_000, rays_shadow=12_000_000,
                      shadow_node_visits=50_000_000, shadow_prim_tests=9_000_000, hits_primary=4_000_000,
                      hits_bounce=7_000_000)
HBM = {"node_bytes": 64 * 1000, "num_nodes": 1000, "tri_bytes": 480_000_000, "sphere_bytes": 16 * 8,
       "prim_ref_bytes": 40_000_000, "lds_bytes": 0}
LDS = dict(HBM, tri_bytes=48 * 12, prim_ref_bytes=80, node_bytes=64 * 20, num_nodes=20, lds_bytes=2084)


@pytest.mark.parametrize("layout", [HBM, LDS], ids=["hbm", "lds"])
def test_frac_independent_of_timed_steps(bench, layout):
    a = bench.roofline(CNT, [_step_stats(1)], layout, "no_such_workload", 1)
    b = bench.roofline(CNT, [_step_stats(20)], layout, "no_such_workload", 20)
    s8d = "frac_s8d" if layout is HBM else "s8d_lds_frac"
    for k in ("frac", s8d, "bytes_per_launch", "avg_launch_us", "launches_per_step", "traversed_rays_per_launch"):
        assert a[k] == pytest.approx(b[k], rel=1e-9), k
    sa = bench.shadow_roofline(CNT, [_step_stats(1)], layout, "no_such_workload", 1)
    sb = bench.shadow_roofline(CNT, [_step_stats(20)], layout, "no_such_workload", 20)
    assert sa["frac"] == pytest.approx(sb["frac"], rel=1e-9)


def _stream(tp, tb, hp, hb, env=0.0):
    return tp * (hp * 12.0 + (1 - hp) * (16.0 + env)) + tb * (32.0 + hb * 12.0 + (1 - hb) * (48.0 + env))


def test_bytes_follow_s8d(bench):
    """hbm residency: every visit charged; the ray streams by hit and miss; frac_s8d the
    literal SURVEY.md §8(d) figure (36 B per ray)."""
    r = bench.roofline(CNT, [_step_stats(3)], HBM, "no_such_workload", 3)
    tp, tb = CNT.traced_primary, CNT.traced_bounce
    scene = 64.0 * CNT.node_visits + 48.0 * CNT.tri_tests + 16.0 * CNT.sphere_tests
    per_launch = (_stream(tp, tb, 0.4, 0.25) + scene) / 6
    assert r["bytes_per_launch"] == pytest.approx(per_launch, rel=1e-6)
    assert r["frac"] == pytest.approx(per_launch / 0.3e-3 / 1e9 / 8000.0, rel=1e-3)
    s8d = (36.0 * (tp + tb) + scene) / 6
    assert r["frac_s8d"] == pytest.approx(s8d / 0.3e-3 / 1e9 / 8000.0, rel=1e-3)
    assert r["per_ray"]["primary"]["nodes"] == pytest.approx(3.0)
    assert r["per_ray"]["bounce"]["nodes"] == pytest.approx(60.0 / 28.0, rel=1e-3)


def test_culled_rays_not_charged(bench):
    """Fewer traversed camera rays (more culling) at the same launch time: fewer bytes, lower frac."""
    a = bench.roofline(CNT, [_step_stats(2)], HBM, "no_such_workload", 2)
    b = bench.roofline(CNT, [_step_stats(2, tp=5_000_000)], HBM, "no_such_workload", 2)
    assert b["bytes_per_launch"] < a["bytes_per_launch"]


def test_lds_scene_charges_stream_only(bench):
    r = bench.roofline(CNT, [_step_stats(1)], LDS, "no_such_workload", 1)
    assert r["scene_residency"] == "lds"
    # §8(d)'s node/primitive bytes of an LDS-staged scene are priced against the LDS roof, never HBM
    assert "frac_s8d" not in r
    s8d = (36.0 * (CNT.traced_primary + CNT.traced_bounce) + 64.0 * CNT.node_visits + 48.0 * CNT.tri_tests
           + 16.0 * CNT.sphere_tests) / 6
    assert r["s8d_lds_frac"] == pytest.approx(s8d / 0.3e-3 / 1e9 / 150000.0, rel=1e-3)
    assert r["bytes_per_launch"] == pytest.approx(_stream(CNT.traced_primary, CNT.traced_bounce, 0.4, 0.25) / 6,
                                                  rel=1e-6)
    # a cubemap environment: 64 B per miss, up to one copy of the faces per XCD per launch
    c = bench.roofline(CNT, [_step_stats(1)], LDS, "no_such_workload", 1, env_bytes=1 << 30)
    assert c["bytes_per_launch"] == pytest.approx(
        _stream(CNT.traced_primary, CNT.traced_bounce, 0.4, 0.25, env=64.0) / 6, rel=1e-6)
    d = bench.roofline(CNT, [_step_stats(1)], LDS, "no_such_workload", 1, env_bytes=1000)
    assert d["bytes_per_launch"] == pytest.approx(
        _stream(CNT.traced_primary, CNT.traced_bounce, 0.4, 0.25) / 6 + 8 * 1000, rel=1e-6)


def test_no_shadow_launches_no_entry(bench):
    st = _step_stats(1)
    st.shadow_launches = 0
    assert bench.shadow_roofline(CNT, [st], HBM, "no_such_workload", 1) is None


@pytest.mark.parametrize("tag,wl", [("r03za", "c2"), ("r03za", "c4"), ("r03zf", "c3"), ("r03zf", "c5"),
                                    ("r04p", "c2"), ("r04p", "c4"), ("r04p", "c5"), ("r04q", "c2"), ("r04q", "c4"), ("r04q", "c5"),
                                    ("r04z", "c2"), ("r04z", "c4"), ("r04z", "c5")])
def test_committed_lines_recompute_from_kernel_stats(tag, wl):
    """Each committed bench line's roofline fraction recomputes from the rocprofv3 kernel statistics of
    the same session (tools/recompute_roofline.py: the timed-path instantiations pooled over their
    launches): within 5 % for LDS scenes; within 10 % where the library overlaps launches on a second
    stream (C3, C5), whose durations depend on what ran beside them in each run.  From r04 on, the
    overlapped lines carry roofline_serial (the one-stream pass, recomputed from its own kernel
    statistics), and the overlapped shadow span, which includes the time its launch waits for CUs the
    trace holds, is not compared."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("recompute_roofline", os.path.join(root, "tools", "recompute_roofline.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    serial = os.path.join(root, "profiles", f"{tag}_kernel_stats_{wl}_serial.csv")
    out = mod.recompute(os.path.join(root, "profiles", f"{tag}_bench_{wl}.json"),
                        os.path.join(root, "profiles", f"{tag}_kernel_stats_{wl}.csv"),
                        serial if os.path.exists(serial) else None)
    tol = 0.05 if wl in ("c2", "c4") else 0.10
    assert "roofline" in out
    if tag >= "r04" and wl in ("c3", "c5"):
        assert "roofline_serial.trace" in out and "roofline_serial.shadow" in out
        out.pop("shadow_roofline")
    for key, r in out.items():
        assert key == "step_roofline" or r["stats_launches"] > 0, key
        assert r["rel_diff"] <= tol, (key, r)


def _full_stats(steps, tail=3_000_000, samples=40_000_000):
    st = _step_stats(steps)
    st.rays_tail = tail * steps
    st.samples = samples * steps
    st.waves = 2 * steps
    return st


@pytest.mark.parametrize("layout,env", [(HBM, 0), (LDS, 1 << 30), (LDS, 25 << 20)], ids=["hbm", "lds-cube", "lds-cube-mall"])
def test_step_roofline_components(bench, layout, env):
    """step_roofline: every kernel's modelled bytes per step over the step time; independent of the
    number of timed steps; components as DESIGN.md §4 states them."""
    rf = bench.roofline(CNT, [_step_stats(4)], layout, "no_such_workload", 4, env_bytes=env)
    sh = bench.shadow_roofline(CNT, [_step_stats(4)], layout, "no_such_workload", 4)
    a = bench.step_roofline(CNT, [_full_stats(4)], 4, 3.0, rf, sh, 2_000_000, 16, env_bytes=env)
    b = bench.step_roofline(CNT, [_full_stats(1)], 1, 3.0, rf, sh, 2_000_000, 16, env_bytes=env)
    assert a == b
    parts = a["bytes_by_kernel"]
    assert sum(parts.values()) == pytest.approx(a["bytes_per_step"], abs=len(parts))
    assert parts["trace"] == pytest.approx(rf["bytes_per_launch"] * 6, rel=1e-6)
    assert parts["shadow"] == pytest.approx(sh["bytes_per_launch"] * 6, rel=1e-6)
    hits = 10_000_000 * 0.4 + 28_000_000 * 0.25
    assert parts["shade"] == pytest.approx(hits * (140.0 + 32.0), rel=1e-6)
    culled = 40_000_000 - 10_000_000
    texels = min(64.0 * culled, 8 * env * 2)  # two k_sky launches (sample batches) per step
    assert parts["sky"] == pytest.approx(texels + culled / 16 * 32.0, rel=1e-6)
    assert parts["accum"] == pytest.approx(2_000_000 * 39.0 + 10_000_000 * 16.0, rel=1e-6)
    if layout is HBM:
        assert parts["tail"] == pytest.approx(3_000_000 * rf["scene_hbm_bytes_per_bounce_ray"], rel=1e-6)
        assert rf["scene_hbm_bytes_per_bounce_ray"] > 0
    else:
        assert parts["tail"] == 0
    assert a["frac"] == pytest.approx(a["bytes_per_step"] / 3e-3 / 1e9 / 8000.0, rel=1e-3)


def test_handed_off_walk_bytes_not_charged(bench):
    """hbm residency: the visits k_strag made for handed-off rays (sptr_stats.strag_visits, every call)
    leave the trace launch's bytes; l2/lds scenes (no hand-off) are unaffected."""
    base = bench.roofline(CNT, [_step_stats(2)], HBM, "no_such_workload", 2)
    st = _step_stats(2)
    st.strag_visits = (1_000_000, 200_000, 10_000)
    st.paths_handed_off = 5000
    r = bench.roofline(CNT, [st], HBM, "no_such_workload", 2)
    cut = (64.0 * 1_000_000 + 48.0 * 200_000 + 16.0 * 10_000) / 12
    assert r["bytes_per_launch"] == pytest.approx(base["bytes_per_launch"] - cut, abs=1)
    assert r["handed_off"]["resumed_walk_bytes_per_launch"] == round(cut)
    l = bench.roofline(CNT, [st], LDS, "no_such_workload", 2)
    assert l["handed_off"]["resumed_walk_bytes_per_launch"] == 0
