"""On-disk formats (…_amd/formats.py), CPU only.

Euler conventions are pinned against hand-built rotation matrices: the reference's log_rot2euler
is pymo's expmap2euler = transforms3d axangle2euler(axis, theta, 'rxyz') (rotating axes x, y, z:
R = Rx(a) Ry(b) Rz(c)); transforms3d is not installed here, so the convention is restated and
checked on matrices built from that definition."""
import json
import os
import pickle

import numpy as np
import pytest
import torch as th

from tests.conftest import ROOT  # noqa: F401


@pytest.fixture(scope="module")
def fm(pkg):
    import importlib
    return importlib.import_module(pkg.__name__ + ".formats")


def _rx(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[1, 0, 0], [0, c, -s], [0, s, c]])


def _ry(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])


def _rz(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


def _log_map(R):
    """Rodrigues inverse (rotation angle < pi)."""
    th_ = np.arccos(np.clip((np.trace(R) - 1) / 2, -1, 1))
    if th_ < 1e-12:
        return np.zeros(3)
    w = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]]) / (2 * np.sin(th_))
    return w * th_


def test_log_rot_to_euler_rotating_xyz(fm):
    rng = np.random.RandomState(0)
    angles = np.concatenate([rng.uniform(-80, 80, (20, 3)), [[0, 0, 0], [90, 0, 0], [0, 30, 0], [0, 0, -45]]])
    logs = np.stack([_log_map(_rx(np.radians(a)) @ _ry(np.radians(b)) @ _rz(np.radians(c))) for a, b, c in angles])
    got = fm.log_rot_to_euler(logs.reshape(2, -1))   # (..., 3 J) layout, J = 12 per row
    assert np.allclose(got.reshape(-1, 3), angles, atol=1e-6)
    assert np.allclose(fm.euler_to_log_rot(angles), logs, atol=1e-9)
    assert np.allclose(fm.log_rot_to_euler(np.full((1, 3), 1e-12)), 0.0)   # pymo: theta < 1e-10 -> identity


def test_ortho6d_to_euler(fm):
    R = _rx(0.3) @ _ry(-0.7) @ _rz(1.1)
    six = (R[:, :2] * np.array([2.0, 0.5])).reshape(1, 6)   # column scale is removed by Gram-Schmidt
    assert np.allclose(fm.ortho6d_to_euler(six), np.degrees([[0.3, -0.7, 1.1]]), atol=1e-6)


def test_pose_scaler_inverse_matches_sklearn(fm, tmp_path):
    from sklearn.preprocessing import StandardScaler
    x = np.random.RandomState(1).randn(200, 9) * 3 + 2
    sk = StandardScaler().fit(x)
    ps = fm.PoseScaler.from_sklearn(sk)
    y = sk.transform(x[:7]).reshape(1, 7, 9)
    assert np.allclose(ps.inverse_transform(y), sk.inverse_transform(y[0])[None])
    assert np.allclose(ps.transform(x[:7]), sk.transform(x[:7]))
    ps.save_npz(tmp_path / "scaler.npz")
    conv = fm.PoseTypeConverter(str(tmp_path / "scaler.npz"))
    assert np.allclose(conv.scaled_euler_to_euler(y), ps.inverse_transform(y))
    with pytest.raises(ValueError):
        conv.to_euler(y, "quat")


def test_pose2bvh_layout_and_filter(fm, tmp_path):
    hierarchy = ["HIERARCHY\n", "ROOT Hips\n", "{\n", "  OFFSET 0 0 0\n", "}\n"]
    pose = np.random.RandomState(2).uniform(-30, 30, (50, 6))
    p = tmp_path / "a.bvh"
    fm.pose2bvh(str(p), pose, hierarchy, fps=20, root_translation=[1, 2, 3])
    lines = open(p).read().splitlines()
    assert lines[:5] == [h.rstrip("\n") for h in hierarchy]
    assert lines[5:8] == ["MOTION", "Frames: 50", "Frame Time: 0.05"]
    rows, ft = fm.read_bvh_motion(str(p))
    assert ft == 0.05 and rows.shape == (50, 9)
    assert np.allclose(rows[:, :3], [1, 2, 3]) and np.allclose(rows[:, 3:], pose)
    # the low-pass option keeps a smooth track (its own filter applied twice is stable)
    smooth = np.tile(np.linspace(-10, 10, 50)[:, None], (1, 6))
    fm.pose2bvh(str(tmp_path / "b.bvh"), smooth, hierarchy, filter=True)
    rows, _ = fm.read_bvh_motion(str(tmp_path / "b.bvh"))
    assert np.allclose(rows[:, 3:], smooth, atol=0.5)


def test_checkpoint_dict_roundtrip_into_the_sampler_model(pkg, fm, beat_cfg, tmp_path):
    arch = pkg.arch_from_config(beat_cfg.Model, 123)
    sd = pkg.init_state_dict(arch, seed=3)
    ck = {"model_state_dict": sd, "best_state_dict": sd, "optimizer_state_dict": {"step": 5},
          "lr_scheduler_state_dict": {"last_epoch": 5}, "train_step": 5, "epochs_run": 1,
          "wandb_id": "x", "best_metric_value": 0.5}
    path = tmp_path / "chkpts" / "chkpt_gpu0_seed0.pt"
    os.makedirs(path.parent)
    th.save(ck, path)
    model, _, _, _, _ = pkg.create_model(123, beat_cfg.Model)
    fm.load_model_checkpoint(model, str(path))            # main.py:113-115
    got = model.state_dict()
    assert set(got) == set(sd) and all(th.equal(got[k], sd[k]) for k in sd)
    assert fm.model_state_dict(sd) is sd                  # a bare state_dict passes through


def test_result_files(fm, tmp_path):
    out = np.random.RandomState(4).randn(3, 40, 6).astype(np.float32)
    gen = fm.save_eval_results(str(tmp_path / "results"), {"mse": 0.25, "total_bpd": 1.5}, out,
                               th.from_numpy(out * 2), th.zeros(3, 100))
    with open(tmp_path / "results" / "eval_results.json") as f:
        assert json.load(f) == {"test/mse": 0.25, "test/total_bpd": 1.5}
    with open(tmp_path / "results" / "generated.pkl", "rb") as f:   # our own file
        g = pickle.load(f)
    assert set(g) == {"out", "pose", "wav"} and np.array_equal(g["out"], out) and g["wav"].shape == (3, 100)
    ps = fm.PoseScaler(np.zeros(6), np.ones(6))
    logs = np.random.RandomState(5).uniform(-1, 1, (2, 40, 6))
    paths = fm.save_samples(str(tmp_path / "samples"), [logs[0], logs[1]], [logs[1], logs[0]], [np.zeros(10)] * 2,
                            fm.PoseTypeConverter(ps), "log_rot")
    assert [os.path.basename(p) for p in paths] == ["sample_0.pkl", "sample_1.pkl"]
    with open(paths[1], "rb") as f:
        s1 = pickle.load(f)
    assert np.allclose(s1["out"], fm.log_rot_to_euler(logs[1])) and np.allclose(s1["pose"], fm.log_rot_to_euler(logs[0]))
