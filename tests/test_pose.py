"""Row A23: tag pose + the node's camera->robot transform and distance sort.

CPU tests: the oracle's estimate_tag_pose restatement (oracle/ao_pose.c)
against exact ground truth, and the host tail at_tag_detections against the
reference's own test cases (test/coordinate_transform_test.cu,
test/detection_sorting_test.cu).  The GPU pose (k_pose) is compared with the
oracle in tests/test_gpu_parity.py.  Parity of the restatement with the
upstream AprilTag library itself is unpinned (no pose fixture exists in the
reference).
"""
import math

import numpy as np
import pytest

FX, FY, CX, CY, TS = 905.495617, 907.909470, 609.916016, 352.682645, 0.1651


def _rot(ax, ay, az):
    cx, sx, cy, sy, cz, sz = math.cos(ax), math.sin(ax), math.cos(ay), math.sin(ay), math.cos(az), math.sin(az)
    Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def _project(R, t):
    """Homography tag [-1,1]^2 -> pixels and the detection corner order
    p[i] = H*(-1,1),(1,1),(1,-1),(-1,-1) of apriltag_detection_t."""
    K = np.array([[FX, 0, CX], [0, FY, CY], [0, 0, 1]])
    s = TS / 2
    H = K @ np.column_stack([R[:, 0] * s, R[:, 1] * s, t])
    H /= H[2, 2]
    corners = np.array([(H @ [x, y, 1])[:2] / (H @ [x, y, 1])[2] for x, y in [(-1, 1), (1, 1), (1, -1), (-1, -1)]])
    return H, corners


def test_oracle_pose_recovers_exact_projection(oracle_mod):
    rng = np.random.default_rng(766)
    for _ in range(100):
        R = _rot(*rng.uniform(-0.7, 0.7, 3))
        t = np.array([rng.uniform(-0.6, 0.6), rng.uniform(-0.3, 0.3), rng.uniform(0.6, 5.0)])
        H, corners = _project(R, t)
        Re, te, err, _, _ = oracle_mod.estimate_tag_pose(H, corners, FX, FY, CX, CY, TS)
        assert np.abs(Re - R).max() < 1e-9
        assert np.abs(te - t).max() < 1e-9
        assert err < 1e-18


def test_oracle_pose_noisy_corners_is_a_rotation_and_picks_smaller_error(oracle_mod):
    rng = np.random.default_rng(1)
    seen_second = 0
    for _ in range(150):
        R = _rot(*rng.uniform(-0.9, 0.9, 3))
        t = np.array([rng.uniform(-0.5, 0.5), rng.uniform(-0.3, 0.3), rng.uniform(2.0, 6.0)])
        H, corners = _project(R, t)
        corners = corners + rng.normal(0, 0.5, corners.shape)
        Re, te, err, (e1, e2), second = oracle_mod.estimate_tag_pose(H, corners, FX, FY, CX, CY, TS)
        assert np.abs(Re @ Re.T - np.eye(3)).max() < 1e-12
        assert abs(np.linalg.det(Re) - 1) < 1e-12
        assert err == min(e1, e2)
        assert second == (not e1 <= e2)
        assert te[2] > 0  # in front of the camera
        seen_second += second
    assert seen_second > 0  # the fix_pose_ambiguities branch is exercised


# ---- the node's host tail: transformCameraToRobot + distance sort ----------

def _pose(tid, t):
    from ros_vision_amd.detector import Pose
    return Pose(id=tid, R=np.eye(3), t=np.asarray(t, np.float64), err=0.01 * tid)


def _rz(a):
    return np.array([[math.cos(a), -math.sin(a), 0], [math.sin(a), math.cos(a), 0], [0, 0, 1]])


@pytest.mark.parametrize("cam,R,off,expect", [
    # coordinate_transform_test.cu: identity, translation only, 90 deg about Z, 45 deg + offset, zero input
    ((1.0, 2.0, 3.0), np.eye(3), (0, 0, 0), (1.0, 2.0, 3.0)),
    ((1.0, 2.0, 3.0), np.eye(3), (0.5, -0.25, 1.0), (1.5, 1.75, 4.0)),
    ((1.0, 0.0, 0.0), _rz(math.pi / 2), (0, 0, 0), (0.0, 1.0, 0.0)),
    ((1.0, 0.0, 0.0), _rz(math.pi / 4), (0.5, -0.5, 1.0),
     (math.sqrt(2) / 2 + 0.5, math.sqrt(2) / 2 - 0.5, 1.0)),
    ((0.0, 0.0, 0.0), _rz(math.pi / 4), (0.5, -0.5, 1.0), (0.5, -0.5, 1.0)),
])
def test_camera_to_robot_transform(cam, R, off, expect):
    from ros_vision_amd.detector import tag_detections
    (o,) = tag_detections([_pose(7, cam)], R, off)
    assert np.allclose(o.robot, expect, atol=1e-9)
    assert np.allclose(o.camera, cam)
    assert o.distance == pytest.approx(math.sqrt(sum(c * c for c in cam)), abs=1e-12)


def test_rotation_preserves_distance():
    from ros_vision_amd.detector import tag_detections
    (o,) = tag_detections([_pose(1, (3.0, 4.0, 0.0))], _rz(0.7), None)
    assert np.linalg.norm(o.robot) == pytest.approx(5.0, abs=1e-12)


def test_sorted_closest_first():
    """detection_sorting_test.cu SortingOrderCorrectness: ids 1,2,3 at 5,2,1 m -> 3,2,1."""
    from ros_vision_amd.detector import tag_detections
    out = tag_detections([_pose(1, (3.0, 4.0, 0.0)), _pose(2, (0.0, 0.0, 2.0)), _pose(3, (1.0, 0.0, 0.0))])
    assert [o.id for o in out] == [3, 2, 1]
    assert [o.distance for o in out] == pytest.approx([1.0, 2.0, 5.0])
    assert [o.err for o in out] == pytest.approx([0.03, 0.02, 0.01])


def test_sort_edge_cases():
    """SortingEdgeCases + SortingEqualDistances + SortingPerformance."""
    from ros_vision_amd.detector import tag_detections
    assert tag_detections([]) == []
    assert [o.id for o in tag_detections([_pose(1, (1.0, 1.0, 1.0))])] == [1]
    eq = tag_detections([_pose(1, (1.0, 0.0, 0.0)), _pose(2, (0.0, 1.0, 0.0))])
    assert [o.id for o in eq] == [1, 2]  # equal distances keep their order
    many = tag_detections([_pose(i, (1000.0 - i, 0.0, 0.0)) for i in range(1000)])
    d = [o.distance for o in many]
    assert d == sorted(d) and many[0].id == 999
