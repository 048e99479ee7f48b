"""CPU: the densification oracle (oracle/strategy_oracle.py) against goldens
produced by the reference's own DefaultStrategy._grow_gs / _prune_gs /
reset_opa with torch.optim.Adam (tests/golden/make_golden_strategy.py).

Bars: the counts, the surviving rows' order and every copied value are exact;
the split children's means (a 3x3 product the reference evaluates with
torch.einsum), log-scales and -- with revised_opacity -- opacity logits
(transcendentals of another libm) within a few fp32 ulps."""

import numpy as np
import pytest

from conftest import load_golden
from oracle import strategy_oracle as S

NAMES = ("means", "scales", "quats", "opacities", "sh0", "shN")
CASES = ["densify_early", "densify_late", "densify_revised", "densify_reset", "densify_scale2d"]


def golden_inputs(g):
    params = {k: g[f"in_{k}"] for k in NAMES}
    moments = {k: (g[f"in_m_{k}"], g[f"in_v_{k}"]) for k in NAMES}
    return params, moments


def check_against_golden(g, params, moments, counts=None):
    if counts is not None:
        assert counts == (int(g["n_dupli"]), int(g["n_split"]), int(g["n_prune"]))
    for k in NAMES:
        ref = g[f"out_{k}"]
        got = np.asarray(params[k])
        assert got.shape == ref.shape, (k, got.shape, ref.shape)
        if k in ("means", "scales") or (k == "opacities" and int(g["revised"])):
            np.testing.assert_allclose(got, ref, rtol=2e-6, atol=1e-6, err_msg=k)
        else:
            np.testing.assert_array_equal(got, ref, err_msg=k)
        np.testing.assert_array_equal(np.asarray(moments[k][0]), g[f"out_m_{k}"], err_msg=k)
        np.testing.assert_array_equal(np.asarray(moments[k][1]), g[f"out_v_{k}"], err_msg=k)


@pytest.mark.parametrize("name", CASES)
def test_refine_oracle_matches_reference(name):
    g = load_golden(name)
    params, moments = golden_inputs(g)
    p, m, counts = S.refine(params, moments, g["grad2d"], g["count"], int(g["step"]), g["z"],
                            scene_scale=float(g["scene_scale"]),
                            revised_opacity=bool(g["revised"]), radii2d=g.get("radii2d"))
    if int(g["reset"]):
        p, m = S.reset_opacity(p, m, 0.01)
    check_against_golden(g, p, m, counts)
