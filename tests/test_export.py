"""brax JSON / HTML trajectory export, CPU only.

Pinned against the reference's own artefact: the brax ``Config`` embedded in
``notebooks/ant_tag.ipynb:449`` (fixture tests/golden/ant_tag_notebook_trajectory.json).
That config is the legacy-spring one of an older AntTag (capsule walls at +-7), so the
comparison covers what both share: the ant's bodies, joints (minus the legacy spring
fields), actuators, the Ground and Target bodies, the ground contact pairs and the global
physics scalars.  The box walls are checked against SURVEY.md Appendix A (from
envs/utils.py).
"""
import ctypes as C
import json
import math
import os

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def nb_config():
    return json.load(open(os.path.join(HERE, "golden", "ant_tag_notebook_trajectory.json")))["config"]


def _params():
    from po_brax_amd import _lib
    p = _lib.pob_params()
    assert _lib.lib.pob_default_params(C.byref(p)) == 0
    return p


def test_ant_part_matches_notebook_config(nb_config):
    from po_brax_amd.io.config import brax_config_of
    cfg = brax_config_of("ant_tag", _params())
    names = [b["name"] for b in cfg["bodies"]]
    assert names[:11] == [b["name"] for b in nb_config["bodies"][:11]]  # ant, Ground, Target
    for mine, ref in zip(cfg["bodies"][:11], nb_config["bodies"][:11]):
        assert mine == ref, mine["name"]
    legacy = {"stiffness", "springDamping"}
    assert cfg["joints"] == [{k: v for k, v in j.items() if k not in legacy} for j in nb_config["joints"]]
    assert cfg["actuators"] == nb_config["actuators"]
    assert cfg["collideInclude"][:5] == nb_config["collideInclude"][:5]
    assert cfg["collideInclude"] == nb_config["collideInclude"]  # same Ant x Arena pairs
    for k in ("friction", "gravity", "angularDamping", "dt", "substeps", "frozen", "forces", "elasticity",
              "velocityDamping", "colliderCutoff", "meshGeometries", "defaults"):
        assert cfg[k] == nb_config[k], k
    assert cfg["dynamicsMode"] == "pbd" and "baumgarteErp" not in cfg


def test_box_walls_match_utils(nb_config):
    from po_brax_amd.io.config import brax_config_of
    cfg = brax_config_of("ant_heavenhell", _params())
    arena = cfg["bodies"][-1]
    assert arena["name"] == "Arena" and len(arena["colliders"]) == 8
    # SURVEY.md Appendix A, HH (draw_t_maze(6.25, 8, 2, .5)): centre, rot, halfsize
    want = [((0, 8.5), 0, (6.75, .5, .5)), ((6.75, 7), 90, (1.5, .5, .5)), ((4.625, 5.5), 180, (2.125, .5, .5)),
            ((2.5, 2.5), 90, (3, .5, .5)), ((0, -.5), 180, (2.5, .5, .5)), ((-2.5, 2.5), 90, (3, .5, .5)),
            ((-4.625, 5.5), 180, (2.125, .5, .5)), ((-6.75, 7), 90, (1.5, .5, .5))]
    for c, (xy, rz, hs) in zip(arena["colliders"], want):
        assert (c["position"]["x"], c["position"]["y"]) == pytest.approx(xy)
        # acos gives the unsigned angle: 90 for both vertical walls (envs/utils.py:23)
        assert c["rotation"]["z"] == pytest.approx(rz, abs=1e-4)
        assert (c["box"]["halfsize"]["x"], c["box"]["halfsize"]["y"], c["box"]["halfsize"]["z"]) == pytest.approx(hs)
    tag = brax_config_of("ant_tag", _params())["bodies"][-1]["colliders"]
    assert [(c["position"]["x"], c["position"]["y"]) for c in tag] == [(5.75, 0.0), (0.0, -5.75), (-5.75, 0.0), (0.0, 5.75)]
    ga = brax_config_of("ant_gather", _params())
    assert [b["name"] for b in ga["bodies"][10:]] == (["Arena"] + [f"Target_{i}" for i in range(1, 9)]
                                                     + [f"Bomb_{i}" for i in range(1, 9)])
    assert [b["name"] for b in brax_config_of("ant", _params())["bodies"]][-1] == "Ground"


def test_json_and_html_round_trip():
    from po_brax_amd.envs.env import QP
    from po_brax_amd.io import html, json as bjson
    from po_brax_amd.io.config import brax_config_of

    class FakeEnv:  # the export reads kind / params / action_repeat only
        kind, _params, _action_repeat = "ant_tag", _params(), 1

        @property
        def unwrapped(self):
            return self

    g = torch.Generator().manual_seed(0)
    qps = [QP(torch.rand((4, 12, 3), generator=g), torch.rand((4, 12, 4), generator=g).half(), None, None)
           for _ in range(3)]
    d = json.loads(bjson.dumps(FakeEnv(), qps, env_index=2))
    assert d["config"] == json.loads(json.dumps(brax_config_of("ant_tag", _params())))
    np.testing.assert_array_equal(np.array(d["pos"], np.float32), torch.stack([q.pos[2] for q in qps]).numpy())
    np.testing.assert_array_equal(np.array(d["rot"], np.float32), torch.stack([q.rot[2].float() for q in qps]).numpy())
    page = html.render(FakeEnv(), qps, height=320, env_index=2)
    start = page.index("var system = ") + len("var system = ")
    obj, _ = json.JSONDecoder().raw_decode(page[start:])
    assert obj == d
    assert "height: 320px" in page and "viewer.js" in page
    assert math.isfinite(d["config"]["dt"])
