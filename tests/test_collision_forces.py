"""Contact forces: the reference's World.get_entity_collision_force /
get_wall_collision_force have no caller (core.py:741-836), so the rollout never applies them; the
optional kernel phase (lsm_config.collision_forces) reports them. CPU side: the oracle's
restatement pinned to golden vectors recorded by calling the reference's own functions
(tests/golden/make_golden.py record_collision_forces)."""
import os

import numpy as np

from oracle.lsm_oracle import (CONTACT_FORCE, CONTACT_MARGIN, ENTITY_SIZE, WALL_CONTACT_FORCE,
                               WALL_CONTACT_MARGIN, entity_collision_force, wall_collision_force)

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "collision_forces.npz")


def test_constants_match_reference():
    z = np.load(GOLD)
    assert float(z["contact_force"]) == CONTACT_FORCE and float(z["contact_margin"]) == CONTACT_MARGIN
    assert float(z["wall_contact_force"]) == WALL_CONTACT_FORCE
    assert float(z["wall_contact_margin"]) == WALL_CONTACT_MARGIN
    assert float(z["agent_size"]) == ENTITY_SIZE


def test_entity_collision_force_matches_reference():
    z = np.load(GOLD)
    pos, done, forces = z["pos"], z["done"], z["forces"]
    E = forces.shape[0]
    N = len(pos)
    sizes, collide, movable = z["sizes"], z["collide"], z["movable"]
    # entity positions: agents as placed, landmarks as the reference had them (only agent pairs
    # collide, so landmark positions never enter a non-None force)
    hit = 0
    for a in range(E):
        for b in range(a + 1, E):
            if a < N and b < N:
                d = pos[a] - pos[b]
                dist = np.linalg.norm(np.stack([d]), axis=1)[0]   # cached_dist_mag (norm over axis)
            else:
                d, dist = np.zeros(2), 1.0
            fa, fb = entity_collision_force(d, dist, sizes[a] + sizes[b], bool(done[a]) if a < N else False,
                                            bool(done[b]) if b < N else False, bool(collide[a]), bool(collide[b]),
                                            bool(movable[a]), bool(movable[b]))
            for f, ref in ((fa, forces[a, b, 0]), (fb, forces[a, b, 1])):
                if f is None:
                    assert np.isnan(ref).all(), (a, b)
                else:
                    np.testing.assert_array_equal(f, ref, err_msg="pair %d %d" % (a, b))
                    hit += 1
    assert hit >= 14


def test_wall_collision_force_matches_reference():
    z = np.load(GOLD)
    for wi, w in enumerate(z["walls"]):
        wall = ("H" if w[0] == 0 else "V", float(w[1]), (float(w[2]), float(w[3])), float(w[4]), bool(w[5]))
        for k, p in enumerate(z["wall_pos"]):
            f = wall_collision_force(p, float(z["agent_size"]), wall)
            ref = z["wall_force"][wi, k]
            if f is None:
                assert np.isnan(ref).all()
            else:
                np.testing.assert_array_equal(f, ref, err_msg="wall %d pos %d" % (wi, k))
