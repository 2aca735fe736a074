"""On-disk formats around the sampler.

  checkpoints   the Trainer's dict (trainer.py:200-224: model_state_dict, best_state_dict,
                optimizer_state_dict, lr_scheduler_state_dict, train_step, ...) read back as
                main.py:113-115 does (model.load_state_dict(chkpt["model_state_dict"]));
                torch.load(weights_only=True): tensors and plain containers only
  results       evaluate(): results/eval_results.json and results/generated.pkl {out, pose, wav}
                (main.py:243-267); generate(): results/samples/sample_{i}.pkl {pose, wav, out}
                with the poses converted to euler degrees (main.py:310-334)
  poses         inverse standardisation (the StandardScaler of datasets/dataset.py:72-79: x scale_
                + mean_), log-rotation / 6-D -> euler conversions (the PoseTypeConverter that
                main.py:152-155, 207-214, 317-322 calls and the reference does not ship; designed
                from those call sites and datasets/data_utils.py:71-116), BVH text writer
                (utils/pose2bvh.py:27-53, with its optional low-pass filter :16-24)
"""
import json
import os
import pickle

import numpy as np
import torch as th
from scipy.signal import butter, filtfilt
from scipy.spatial.transform import Rotation


# ------------------------------------------------------------------------------------------
# checkpoints
# ------------------------------------------------------------------------------------------
def load_checkpoint(path, map_location="cpu"):
    """A checkpoint dict written by the reference Trainer (or by training.Trainer.checkpoint)."""
    return th.load(path, map_location=map_location, weights_only=True)


def model_state_dict(ckpt, which="model_state_dict"):
    """main.py:113-115 unwraps chkpt["model_state_dict"]; fine-tuning reads "best_state_dict"
    (model_creation.py:163-166).  A bare state_dict passes through."""
    if isinstance(ckpt, dict) and which in ckpt:
        return ckpt[which]
    return ckpt


def load_model_checkpoint(model, path, which="model_state_dict", strict=True):
    """model.load_state_dict(chkpt[which]) for the HIP sampler model or a TrainableModel."""
    return model.load_state_dict(model_state_dict(load_checkpoint(path), which), strict=strict)


def save_checkpoint(path, trainer, best_state_dict=None, epochs_run=0, best_metric_value=float("inf"), wandb_id=""):
    """The reference's checkpoint layout (trainer.py:200-212) from a training.Trainer."""
    ck = trainer.checkpoint()
    ck.update({"best_state_dict": best_state_dict if best_state_dict is not None else ck["model_state_dict"],
               "epochs_run": epochs_run, "wandb_id": wandb_id, "best_metric_value": best_metric_value})
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    th.save({k: _cpu(v) for k, v in ck.items()}, path)


def _cpu(v):
    if isinstance(v, th.Tensor):
        return v.detach().cpu()
    if isinstance(v, dict):
        return {k: _cpu(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_cpu(x) for x in v]
    return v


# ------------------------------------------------------------------------------------------
# pose conversions
# ------------------------------------------------------------------------------------------
class PoseScaler:
    """sklearn StandardScaler's transform / inverse_transform from its mean_ and scale_
    (datasets/dataset.py:72-79 fits it on (N T, d_pose) poses)."""

    def __init__(self, mean, scale):
        self.mean_ = np.asarray(mean, dtype=np.float64)
        self.scale_ = np.asarray(scale, dtype=np.float64)

    @classmethod
    def from_sklearn(cls, scaler):
        return cls(scaler.mean_, scaler.scale_)

    @classmethod
    def from_npz(cls, path):
        with np.load(path, allow_pickle=False) as f:
            return cls(f["mean"], f["scale"])

    def save_npz(self, path):
        np.savez(path, mean=self.mean_, scale=self.scale_)

    def transform(self, x):
        x = np.asarray(x)
        return ((x.reshape(-1, x.shape[-1]) - self.mean_) / self.scale_).reshape(x.shape)

    def inverse_transform(self, x):
        x = np.asarray(x)
        return (x.reshape(-1, x.shape[-1]) * self.scale_ + self.mean_).reshape(x.shape)


def log_rot_to_euler(log_rot, seq="XYZ"):
    """datasets/data_utils.py:110-116 log_rot2euler -> pymo expmap2euler (rotation_tools.py:168-179):
    axis-angle (theta = |v|, axis [1, 0, 0] below 1e-10) -> euler degrees about rotating axes x, y, z
    (transforms3d 'rxyz' = scipy's intrinsic 'XYZ').  (..., 3 J) -> (..., 3 J)."""
    v = np.asarray(log_rot, dtype=np.float64)
    flat = v.reshape(-1, 3)
    theta = np.linalg.norm(flat, axis=1)
    flat = np.where(theta[:, None] > 1e-10, flat, 0.0)
    eul = Rotation.from_rotvec(flat).as_euler(seq, degrees=True)
    return eul.reshape(v.shape)


def euler_to_log_rot(euler, seq="XYZ"):
    """datasets/data_utils.py:101-107 euler2log_rot (pymo euler2expmap, degrees)."""
    e = np.asarray(euler, dtype=np.float64)
    return Rotation.from_euler(seq, e.reshape(-1, 3), degrees=True).as_rotvec().reshape(e.shape)


def ortho6d_to_euler(ortho6d, seq="XYZ"):
    """datasets/data_utils.py:71-98: 6-D (two columns of the rotation matrix) -> Gram-Schmidt
    matrix -> euler degrees.  (..., 6 J) -> (..., 3 J)."""
    o = np.asarray(ortho6d, dtype=np.float64)
    m = o.reshape(-1, 3, 2)
    x = m[:, :, 0] / np.maximum(np.linalg.norm(m[:, :, 0], axis=1, keepdims=True), 1e-8)
    z = np.cross(x, m[:, :, 1])
    z = z / np.maximum(np.linalg.norm(z, axis=1, keepdims=True), 1e-8)
    y = np.cross(z, x)
    rot = np.stack([x, y, z], axis=2)
    eul = Rotation.from_matrix(rot).as_euler(seq, degrees=True)
    return eul.reshape(*o.shape[:-1], o.shape[-1] // 2)


def unroll_log_rot(log_rot):
    """Remove the 2 pi jumps of an axis-angle track over frames (T, 3) so it can be filtered
    (the role of data_utils.unroll_log_rot in pose2bvh.py:40): where consecutive vectors point
    apart, switch to the equivalent (theta - 2 pi) representation along the reversed axis."""
    r = np.array(log_rot, dtype=np.float64, copy=True)
    for t in range(1, len(r)):
        th_ = np.linalg.norm(r[t])
        if th_ < 1e-10:
            continue
        alt = r[t] * (1.0 - 2.0 * np.pi / th_)
        if np.linalg.norm(alt - r[t - 1]) < np.linalg.norm(r[t] - r[t - 1]):
            r[t] = alt
    return r


def butter_lowpass_filter(data, cutoff=2, fs=18, order=2):
    """utils/pose2bvh.py:16-24."""
    b, a = butter(order, cutoff / 0.5 / fs, btype="low", analog=False)
    return filtfilt(b, a, data)


class PoseTypeConverter:
    """The converter main.py constructs as PoseTypeConverter(scaler path, hierarchy path)
    (main.py:152-155, 286-289): scaled network poses -> euler degrees (main.py:317-322)."""

    def __init__(self, scaler, hierarchy_path=None):
        self.scaler = scaler if isinstance(scaler, PoseScaler) else PoseScaler.from_npz(scaler)
        self.hierarchy = read_hierarchy(hierarchy_path) if hierarchy_path else None

    def scaled_log_rot_to_euler(self, x):
        return log_rot_to_euler(self.scaler.inverse_transform(x))

    def scaled_ortho6d_to_euler(self, x):
        return ortho6d_to_euler(self.scaler.inverse_transform(x))

    def scaled_euler_to_euler(self, x):
        return self.scaler.inverse_transform(x)

    def to_euler(self, x, representation):
        if representation == "log_rot":
            return self.scaled_log_rot_to_euler(x)
        if representation == "6d":
            return self.scaled_ortho6d_to_euler(x)
        if representation == "euler":
            return self.scaled_euler_to_euler(x)
        raise ValueError(f"Unsupported pose_representation {representation}")


# ------------------------------------------------------------------------------------------
# BVH
# ------------------------------------------------------------------------------------------
def read_hierarchy(path):
    with open(path) as f:
        return f.readlines()


def pose2bvh(bvh_path, pose, hierarchy, fps=20, root_translation=(0, 0, 0), filter=False):
    """utils/pose2bvh.py:27-53: the hierarchy lines, then MOTION / Frames / Frame Time, then one
    row per frame of [root translation, euler angles] (np.savetxt default format)."""
    pose = np.asarray(pose, dtype=np.float64)
    n = pose.shape[0]
    if filter:
        lr = euler_to_log_rot(pose.reshape(-1, 3)).reshape(n, -1, 3)
        lr = np.concatenate([unroll_log_rot(lr[:, j]) for j in range(lr.shape[1])], axis=1)
        filtered = np.array([butter_lowpass_filter(x) for x in lr.T]).T
        pose = log_rot_to_euler(filtered.reshape(-1, 3)).reshape(n, -1)
    motion = np.concatenate([np.repeat(np.asarray(root_translation, dtype=np.float64)[None], n, axis=0), pose], axis=1)
    header = "".join(list(hierarchy) + ["MOTION\n", f"Frames: {n}\n", f"Frame Time: {1 / fps}"])
    np.savetxt(bvh_path, motion, header=header, comments="")


def read_bvh_motion(path):
    """The MOTION block of a BVH written by pose2bvh: (frames, channels) and the frame time."""
    with open(path) as f:
        lines = f.readlines()
    i = next(k for k, l in enumerate(lines) if l.strip() == "MOTION")
    frames = int(lines[i + 1].split(":")[1])
    ft = float(lines[i + 2].split(":")[1])
    rows = np.loadtxt(lines[i + 3:i + 3 + frames], ndmin=2)
    return rows, ft


# ------------------------------------------------------------------------------------------
# result files of main.py's eval / gen phases
# ------------------------------------------------------------------------------------------
def save_eval_results(result_dir, metrics, out, pose, wav):
    """main.py:243-267: results/eval_results.json ({"test/<name>": value}) and results/generated.pkl
    {"out": (N, L, C), "pose": (N, L, C), "wav": (N, T_wav)} numpy arrays."""
    os.makedirs(result_dir, exist_ok=True)
    with open(os.path.join(result_dir, "eval_results.json"), "w") as f:
        json.dump({f"test/{k}": float(v) for k, v in metrics.items()}, f, indent=2)
    gen = {"out": np.asarray(out), "pose": _np(pose), "wav": _np(wav)}
    with open(os.path.join(result_dir, "generated.pkl"), "wb") as f:
        pickle.dump(gen, f)
    return gen


def save_samples(sample_dir, out_seqs, pose_seqs, wav_seqs, converter=None, representation="euler"):
    """main.py:310-334: results/samples/sample_{i}.pkl = {"pose", "wav", "out"} with pose and out
    converted to euler degrees by the PoseTypeConverter (passed through for 'euler')."""
    os.makedirs(sample_dir, exist_ok=True)
    paths = []
    for i, out_seq in enumerate(out_seqs):
        pose_seq = _np(pose_seqs[i])
        out_seq = _np(out_seq)
        if representation != "euler":
            if converter is None:
                raise ValueError("a PoseTypeConverter is needed for " + representation)
            out_seq = converter.to_euler(out_seq, representation)
            pose_seq = converter.to_euler(pose_seq, representation)
        obj = {"pose": pose_seq, "wav": _np(wav_seqs[i]), "out": out_seq}
        p = os.path.join(sample_dir, f"sample_{i}.pkl")
        with open(p, "wb") as f:
            pickle.dump(obj, f)
        paths.append(p)
    return paths


def _np(x):
    return x.detach().cpu().numpy() if isinstance(x, th.Tensor) else np.asarray(x)
