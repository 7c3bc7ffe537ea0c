"""The model's contact-pair table (gym_so100/assets/so100_model.json: 191 pairs, 209 with the EE variant's) against MuJoCo's collision
filters applied to the reference MJCF: the table is exactly the pair set MuJoCo would hand
to a narrowphase, no pair more, none missing.  Filters restated from MuJoCo 3.3.3's broadphase (mj_collision /
filter): contype/conaffinity compatibility, same weld body (which includes static-static), the
parent-child filter (skipped for world-welded bodies), and the model's <exclude> (so_arm100.xml:165-167).
Reads the reference MJCF, so it runs only where /root/reference exists (this container)."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/gym_so100/assets"
pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason="reference MJCF not present")


@pytest.mark.parametrize("variant", ["joint", "ee"])
def test_pair_table_is_mujocos_filtered_pair_set(variant):
    """joint: so100_transfer_cube.xml's pairs (those not marked ee_only); ee: so100_transfer_cube_ee.xml's, the
    same scene plus the mocap body of so_arm100_ee.xml:155 (a jointless child of the world, so welded to it:
    its marker box meets neither the table, the bin nor the Base)."""
    sys.path.insert(0, os.path.join(ROOT, "gym-so100-c_amd", "tools"))
    from compile_model import parse
    _, bodies, _, excludes = parse()
    if variant == "ee":
        bodies = dict(bodies)
        bodies["mocap_target"] = {"joints": [], "parent": "world",
                                  "geoms": [{"name": "mocap_target_box", "type": "box"}]}
    weld = {"world": "world"}

    def weld_of(b):
        if b not in weld:
            weld[b] = b if bodies[b]["joints"] or b == "box" else weld_of(bodies[b]["parent"])
        return weld[b]
    geoms = []
    for bname, rec in bodies.items():
        for g in rec["geoms"]:
            ct, ca = int(g.get("contype", 1)), int(g.get("conaffinity", 1))
            if ct == 0 and ca == 0:
                continue
            geoms.append((bname, g.get("name") or g.get("mesh"), ct, ca))
    want = set()
    for i, (b1, n1, ct1, ca1) in enumerate(geoms):
        for b2, n2, ct2, ca2 in geoms[i + 1:]:
            if not (ct1 & ca2 or ct2 & ca1):
                continue
            w1, w2 = weld_of(b1), weld_of(b2)
            if w1 == w2:
                continue                                   # same weld body, static-static included
            p1 = weld_of(bodies[w1]["parent"]) if w1 != "world" else "world"
            p2 = weld_of(bodies[w2]["parent"]) if w2 != "world" else "world"
            if w1 != "world" and w2 != "world" and (w1 == p2 or w2 == p1):
                continue                                   # parent-child (not for world-welded bodies)
            if (b1, b2) in excludes or (b2, b1) in excludes:
                continue
            want.add(frozenset((n1, n2)))
    model = json.load(open(os.path.join(ROOT, "gym-so100-c_amd", "gym_so100", "assets", "so100_model.json")))
    pairs = [p for p in model["pairs"] if variant == "ee" or not p.get("ee_only")]
    have = {frozenset((p["name1"], p["name2"])) for p in pairs}
    assert len(have) == len(pairs) == {"joint": 191, "ee": 209}[variant]
    assert not have - want, sorted(map(sorted, have - want))     # no pair MuJoCo would filter out
    assert not want - have, sorted(map(sorted, want - have))     # none missing: round 2 added the 36
    # finger-pad / link-hull pairs (4 links for the fixed-jaw pads, Wrist_Pitch_Roll being their parent, 5
    # for the moving-jaw pads)
    pads = [p for p in pairs if p["name1"].endswith(("_pad_1", "_pad_2", "_pad_3", "_pad_4"))
            and p["g2"] < 0]
    assert len(pads) == 36
