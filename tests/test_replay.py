"""The icp4radar node's frame loop without ROS: `icp4radar_replay` (C++, over the
C ABI) reads a dataset folder of radar_pointcloud_<k>.bin scans and writes the node's output files
(output_result.csv, radar/{pcl_info,velocity,icp,icp_map}.txt — src/iterative_closest_point.cpp:150-191,
:325, :701-706, :757-816).  It is checked against the same loop restated over the oracle (ICP, parse,
fitSineRansac, split, LSQ) and the node's stream formats.

Bars: pcl_info.txt and icp.txt identical text (ICP is bit-exact, so every float of T prints the same);
output_result.csv identical text in the 17 ICP columns and the score; velocity and A, b within the
ego-velocity tolerances (the device's parse differs from glibc's by an ulp, tests/test_ego.py).
"""
import os
import subprocess

import numpy as np
import pytest

from icp4r import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPLAY = os.path.join(ROOT, "icp-4dradar_amd", "icp4r", "_lib", "icp4radar_replay")


def test_replay_program_built_and_usage():
    assert os.path.exists(REPLAY), "icp4radar_replay not built (make -C icp-4dradar_amd)"
    r = subprocess.run([REPLAY], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr


def _g(x: float) -> str:
    """std::ostream << double at precision 15, default floatfield (== %.15g)."""
    return "%.15g" % x


def oracle_replay(folder: str, oracle, seed: int):
    """The node's loop (:263-721) over the oracle: returns the expected file contents.  Every frame's
    points are appended to the running clouds, which are cleared only after a registration (:505 vs
    :698-699): an empty scan carries the other cloud's points into the next frame."""
    frames = []
    k = 0
    while True:
        frames.append(synth.read_bin(os.path.join(folder, "data", f"radar_pointcloud_{k}.bin")))
        if not os.path.exists(os.path.join(folder, "data", f"radar_pointcloud_{k + 1}.bin")):
            break
        k += 1
    pcl_info, vel, icp_lines, csv, pairs = [], [], [], [], []
    out_t = 0.0
    acc_src = np.zeros((0, 4), np.float32)
    acc_tgt = np.zeros((0, 4), np.float32)
    for k, curr in enumerate(frames):
        last = frames[k - 1] if k else frames[0]
        pcl_info.append("%g" % (curr.size / 5.0))
        if len(curr):
            f = oracle.ego_features(curr)
            A, b, best, bh, _ = oracle.ego_ransac(f, seed=seed + (k << 32))
            V, _, _ = oracle.ego_split_lsq(f, A, b)
        else:  # no hypotheses; Eigen's products over 0 rows give Vxyz = 0
            A, b, V = 0.0, 0.0, np.zeros(3)
        vel.append(V)
        acc_src = np.concatenate([acc_src, synth.records_to_xyzi(curr)])
        acc_tgt = np.concatenate([acc_tgt, synth.records_to_xyzi(last)])
        if len(acc_src) and len(acc_tgt):
            o = oracle.align(acc_src, acc_tgt, numerics=oracle.NUM_F32)
            pairs.append((k, len(acc_src), len(acc_tgt)))
            T = o["T"].astype(np.float64)
            icp_lines.append(" ".join(_g(v) for v in [T[0, 0], T[0, 1], T[0, 2], T[0, 3], T[1, 0], T[1, 1], T[1, 2],
                                                      T[1, 3], T[2, 0], T[2, 1], T[2, 2], T[2, 3]]))
            csv.append(["%f" % out_t] + ["%f" % v for v in T.reshape(-1)] + ["%f" % o["fitness"], "%f" % A, "%f" % b])
            out_t += 1.0
            acc_src = acc_src[:0]
            acc_tgt = acc_tgt[:0]
    return pcl_info, np.array(vel), icp_lines, csv, pairs


def _run_replay(folder, seed, batch, csv, extra=()):
    args = [REPLAY, str(folder), "--csv", str(csv), "--seed", str(seed)] + (["--batch"] if batch else []) + list(extra)
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    files = {name: open(os.path.join(folder, "radar", name)).read() for name in ("pcl_info.txt", "velocity.txt",
                                                                              "icp.txt", "icp_map.txt")}
    files["csv"] = open(csv).read() if os.path.exists(csv) else None
    return files


def _check_against_oracle(got, folder, oracle_mod, seed, v=None):
    pcl_info, vel, icp_lines, csv_rows, pairs = oracle_replay(str(folder), oracle_mod, seed)
    assert got["pcl_info.txt"].splitlines() == pcl_info
    assert got["icp.txt"].splitlines() == icp_lines
    assert got["icp_map.txt"] == ""
    lines = got["csv"].splitlines()
    assert lines[0].startswith("#time(s),Rtrans00") and len(lines) == 1 + len(csv_rows)
    for row, exp in zip(lines[1:], csv_rows):
        cols = row.split(",")
        assert cols[:18] == exp[:18]  # time, the 16 entries of T, the fitness score
        assert abs(float(cols[18]) - float(exp[18])) < 0.05 and abs(float(cols[19]) - float(exp[19])) < 0.05
    gv = np.array([[float(x) for x in l.split()] for l in got["velocity.txt"].splitlines()])
    assert gv.shape == vel.shape and np.abs(gv - vel).max() < 1e-3
    if v is not None:
        nz = np.abs(vel).sum(1) > 0
        assert np.abs(gv[nz] - (-v)).max() < 0.05  # the known sensor velocity
    return pairs


@pytest.mark.gpu
def test_replay_matches_oracle_loop(tmp_path, oracle_mod):
    frames, v = synth.make_sequence(11, frames=6, n=2048)
    frames[3] = frames[3][:1500]  # ragged scans
    synth.write_sequence(str(tmp_path), frames)
    seed = 77
    outs = {mode: _run_replay(tmp_path, seed, mode == "batch", tmp_path / f"out_{mode}.csv")
            for mode in ("frame", "batch")}
    assert outs["frame"] == outs["batch"]  # one device batch == the per-frame loop, byte for byte
    _check_against_oracle(outs["batch"], tmp_path, oracle_mod, seed, v)
    # the batch sharded over several contexts (icp4r_align_batch_multi; one device here, listed three
    # times: three contexts, three streams, three host threads) — byte-identical
    multi = _run_replay(tmp_path, seed, True, tmp_path / "out_multi.csv", ["--devices", "0,0,0"])
    assert multi == outs["batch"]


@pytest.mark.gpu
@pytest.mark.parametrize("empty", [[3], [0], [2, 3]])
def test_replay_empty_scans_accumulate(tmp_path, oracle_mod, empty):
    """Empty scans (:505 vs :698-699): the frame is skipped, the other cloud keeps its points and the
    next frame's points are appended — e.g. an empty scan 0 makes frame 2 register scan 1 + scan 2
    against scan 1.  Both modes match the loop restated over the oracle."""
    frames, v = synth.make_sequence(12, frames=6, n=1024)
    for k in empty:
        frames[k] = frames[k][:0]
    synth.write_sequence(str(tmp_path), frames)
    seed = 5
    outs = {mode: _run_replay(tmp_path, seed, mode == "batch", tmp_path / f"out_{mode}.csv")
            for mode in ("frame", "batch")}
    assert outs["frame"] == outs["batch"]
    pairs = _check_against_oracle(outs["batch"], tmp_path, oracle_mod, seed, v)
    n = [len(f) for f in frames]
    if empty == [0]:  # frame 0 (0 vs 0) and frame 1 (1 vs empty 0) skipped; frame 2: 1+2 vs 1
        assert pairs[0] == (2, n[1] + n[2], n[1])
    if empty == [3]:  # frame 3 (empty vs 2) skipped; frame 4: 4 vs 2 + empty 3
        assert (4, n[4], n[2]) in pairs and all(p[0] != 3 for p in pairs)


@pytest.mark.gpu
def test_replay_use_icp_result(tmp_path, oracle_mod):
    """USE_ICP_RESULT (:192-206, :523-540): no ICP; each registered frame reads the next row of a
    previous run's output_result.csv (header consumed first; fields 1..16 are Rtrans row-major).  The
    poses in icp.txt are the CSV's values composed, and no CSV is written; rows past the end read as
    zeros."""
    frames, _ = synth.make_sequence(13, frames=6, n=1024)
    frames[2] = frames[2][:0]
    synth.write_sequence(str(tmp_path), frames)
    csv = tmp_path / "first.csv"
    first = _run_replay(tmp_path, 3, True, csv)
    rows = [[float(x) for x in ln.split(",")] for ln in first["csv"].splitlines()[1:]]
    replay_csv = tmp_path / "replay_out.csv"
    got = _run_replay(tmp_path, 3, False, replay_csv, ["--use-icp-result", str(csv)])
    assert got["csv"] is None  # #ifndef USE_ICP_RESULT around the CSV writer
    exp = [" ".join(_g(r[c]) for c in (1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12)) for r in rows]
    assert got["icp.txt"].splitlines() == exp
    assert got["velocity.txt"] == first["velocity.txt"] and got["pcl_info.txt"] == first["pcl_info.txt"]
    # a CSV shorter than the sequence: the missing rows read as zero transforms
    short = tmp_path / "short.csv"
    short.write_text("\n".join(first["csv"].splitlines()[:3]) + "\n")
    got2 = _run_replay(tmp_path, 3, False, tmp_path / "x.csv", ["--use-icp-result", str(short)])
    lines2 = got2["icp.txt"].splitlines()
    assert lines2[:2] == exp[:2] and all(set(l.split()) == {"0"} for l in lines2[2:])
