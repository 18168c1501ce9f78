"""BA beyond the C2/C3 shapes, on the GPU vs the fp64 oracle (1e-4 abs, the
north star's bar):

* high-degree frames (40+ outgoing edges, the backend's max_factors = 16 t
  regime, droid_backend.py:31): the wide Schur path (ba_frame_prep +
  ba_frame_gram_wide), no out-degree limit;
* the C5-shaped global BA (2048 KF / ~16k edges with revisit loops, SURVEY.md
  §8d) on one device: fill-reducing pose order + tile-sparse dataflow
  Cholesky on the 12282-variable reduced system;
* the same BA edge-sharded over 2 ranks (gloo, both on cuda:0): per-rank
  Schur terms, all-reduce of the input tiles, identical solves; and over 4
  ranks (middle-rank partitions) at the config's 48x64 depth maps;
* the failure handling: timeouts and a stale sync area, single-device and
  agreed across ranks.
Most C5 tests use 16x24 depth maps: the graph, not the image, is what C5
scales, and the fp64 oracle then finishes in well under a minute."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from droid_mi355x import synthetic
from gpu_util import dev, host
from oracle import ba as oba

pytestmark = pytest.mark.gpu
TOL = 1e-4
KEYS = ("poses", "disps", "intrinsics", "disps_sens", "targets", "weights", "eta", "ii", "jj", "t0", "t1")
HERE = os.path.dirname(os.path.abspath(__file__))
C5_HW = (16, 24)


def _gpu_ba(prob, iterations, lm, ep, bk=None):
    import droid_backends
    droid_backends = bk or droid_backends
    poses, disps = dev(prob["poses"]), dev(prob["disps"])
    dx, dz = droid_backends.ba(poses, disps, dev(prob["intrinsics"]), dev(prob["disps_sens"]), dev(prob["targets"]),
                               dev(prob["weights"]), dev(prob["eta"]), dev(prob["ii"]), dev(prob["jj"]), prob["t0"],
                               prob["t1"], iterations, lm, ep, False)
    torch.cuda.synchronize()
    return dict(dx=host(dx), dz=host(dz), poses=host(poses), disps=host(disps))


def _check(got, ref, tol=TOL):
    for k in ("dx", "dz", "poses", "disps"):
        np.testing.assert_allclose(got[k], ref[k], atol=tol, rtol=0, err_msg=k)


@pytest.mark.parametrize("out_degree", [24, 42])
def test_ba_high_degree_frames(out_degree):
    import droid_backends
    ii, jj = synthetic.dense_edges(num_kf=48, out_degree=out_degree, rng=np.random.default_rng(out_degree))
    prob = synthetic.ba_problem("X", H=24, W=32, seed=90 + out_degree, edges=(ii, jj), sens_fraction=0.2)
    plan = droid_backends.get_plan(prob["ii"], prob["jj"], 48, 24, 32, 1, 48, prob["eta"].shape[0], False, "cuda:0")
    assert plan.num_wide > 0 and np.bincount(prob["ii"]).max() >= out_degree
    got = _gpu_ba(prob, 2, 1e-4, 0.1)
    ref = oba.ba(**{k: prob[k] for k in KEYS}, iterations=2, lm=1e-4, ep=0.1, motion_only=False)
    _check(got, ref)
    assert np.abs(ref["dx"]).max() > 1e-4


def test_ba_mixed_narrow_and_wide_frames():
    """a C3-like graph where a few hub frames carry 30+ loop edges: both Schur paths in one solve."""
    ii, jj = synthetic.c3_edges(num_kf=64, num_edges=512, rng=np.random.default_rng(5))
    hubs = [10, 40]
    extra = [(h, j) for h in hubs for j in range(64) if abs(h - j) > 3 and j % 2 == 0][:56]
    have = set(zip(ii.tolist(), jj.tolist()))
    extra = [e for e in extra if e not in have]
    ii = np.concatenate([ii, [e[0] for e in extra]]).astype(np.int64)
    jj = np.concatenate([jj, [e[1] for e in extra]]).astype(np.int64)
    prob = synthetic.ba_problem("X", H=24, W=32, seed=95, edges=(ii, jj))
    got = _gpu_ba(prob, 2, 1e-5, 1e-2)
    ref = oba.ba(**{k: prob[k] for k in KEYS}, iterations=2, lm=1e-5, ep=1e-2, motion_only=False)
    _check(got, ref)


@pytest.fixture(scope="module")
def c5():
    prob = synthetic.ba_problem("C5", H=C5_HW[0], W=C5_HW[1])
    ref = oba.ba(**{k: prob[k] for k in KEYS}, iterations=2, lm=1e-5, ep=1e-2, motion_only=False)
    return prob, ref


@pytest.mark.timeout(240)
def test_ba_c5_scale_unsharded(c5):
    import droid_backends
    prob, ref = c5
    assert prob["t1"] - prob["t0"] == 2047 and len(prob["ii"]) >= 15000
    plan = droid_backends.get_plan(prob["ii"], prob["jj"], 2048, C5_HW[0], C5_HW[1], 1, 2048,
                                   prob["eta"].shape[0], False, "cuda:0")
    assert plan.order != "identity"
    got = _gpu_ba(prob, 2, 1e-5, 1e-2)
    _check(got, ref)
    assert np.abs(ref["dx"]).max() > 1e-4


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(300)
def test_ba_c5_sharded_two_ranks(c5, tmp_path):
    prob, ref = c5
    out = str(tmp_path / "c5")
    _torchrun(2, [out, C5_HW[0], C5_HW[1]], 280)
    covered = np.zeros(2048, bool)
    edges = 0
    for rank in range(2):
        d = np.load(out + ".rank%d.npz" % rank)
        lo, hi = (int(x) for x in d["own"])
        edges += int(d["edges"])
        np.testing.assert_allclose(d["dx"], ref["dx"], atol=TOL, rtol=0)
        np.testing.assert_allclose(d["poses"], ref["poses"], atol=TOL, rtol=0)
        np.testing.assert_allclose(d["disps"][lo:hi], ref["disps"][lo:hi], atol=TOL, rtol=0)
        covered[lo:hi] = True
    assert covered.all() and edges == len(prob["ii"])


def test_chol_timeout_is_reported_and_state_untouched(ab_backends):
    """The dataflow solve's safety net (bounded spins -> abort, flag bit 1):
    forced here with the test hook, ba() must raise and leave poses/disps as
    they were (the abort used to corrupt them silently)."""
    droid_backends = ab_backends   # the fault-injection hook ships in the testing builds only
    prob = synthetic.ba_problem("C3", H=16, W=24)
    poses, disps = dev(prob["poses"]), dev(prob["disps"])
    droid_backends.chol_set_fault_inject(droid_backends.CHOL_INJECT_ALL)
    try:
        with pytest.raises(RuntimeError, match="timed out"):
            droid_backends.ba(poses, disps, dev(prob["intrinsics"]), dev(prob["disps_sens"]), dev(prob["targets"]),
                              dev(prob["weights"]), dev(prob["eta"]), dev(prob["ii"]), dev(prob["jj"]), prob["t0"],
                              prob["t1"], 1, 1e-4, 0.1, False)
    finally:
        droid_backends.chol_set_fault_inject(droid_backends.CHOL_INJECT_OFF)
    np.testing.assert_array_equal(host(poses), prob["poses"])
    np.testing.assert_array_equal(host(disps), prob["disps"])
    got = _gpu_ba(prob, 1, 1e-4, 0.1, ab_backends)          # and the next solve on the same plan is clean
    assert np.isfinite(got["dx"]).all()


def test_chol_timeout_in_first_gn_iteration_is_still_reported(ab_backends):
    """the status word used to be cleared by every solve, so a
    timeout in GN iteration 1 of ba(iterations=2) vanished when iteration 2
    succeeded.  The sticky word keeps it: ba() raises."""
    droid_backends = ab_backends   # the fault-injection hook ships in the testing builds only
    prob = synthetic.ba_problem("C3", H=16, W=24, seed=7)
    poses, disps = dev(prob["poses"]), dev(prob["disps"])
    droid_backends.chol_set_fault_inject(droid_backends.CHOL_INJECT_ONCE)
    try:
        with pytest.raises(RuntimeError, match="timed out"):
            droid_backends.ba(poses, disps, dev(prob["intrinsics"]), dev(prob["disps_sens"]), dev(prob["targets"]),
                              dev(prob["weights"]), dev(prob["eta"]), dev(prob["ii"]), dev(prob["jj"]), prob["t0"],
                              prob["t1"], 2, 1e-4, 0.1, False)
    finally:
        droid_backends.chol_set_fault_inject(droid_backends.CHOL_INJECT_OFF)
    got = _gpu_ba(prob, 2, 1e-4, 0.1, ab_backends)          # the next call on the same plan starts clean
    assert np.isfinite(got["dx"]).all()


def test_chol_stale_sync_area_is_detected(ab_backends):
    """the dataflow kernel checks its entry state.  A solve
    launched on a sync area that was not zeroed (the previous launch's ticket
    and version counters) must report status bit 2 and change nothing, not run
    tasks against stale hand-off counters; the solve after it is clean."""
    droid_backends = ab_backends   # the fault-injection hook ships in the testing builds only
    prob = synthetic.ba_problem("C3", H=16, W=24, seed=11)
    ref1 = _gpu_ba(prob, 1, 1e-4, 0.1, ab_backends)          # a clean solve leaves the counters at their final values
    poses, disps = dev(prob["poses"]), dev(prob["disps"])
    droid_backends.chol_set_fault_inject(droid_backends.CHOL_INJECT_STALE)
    try:
        with pytest.raises(RuntimeError, match="state corrupt"):
            droid_backends.ba(poses, disps, dev(prob["intrinsics"]), dev(prob["disps_sens"]), dev(prob["targets"]),
                              dev(prob["weights"]), dev(prob["eta"]), dev(prob["ii"]), dev(prob["jj"]), prob["t0"],
                              prob["t1"], 1, 1e-4, 0.1, False)
    finally:
        droid_backends.chol_set_fault_inject(droid_backends.CHOL_INJECT_OFF)
    np.testing.assert_array_equal(host(poses), prob["poses"])
    np.testing.assert_array_equal(host(disps), prob["disps"])
    got = _gpu_ba(prob, 1, 1e-4, 0.1, ab_backends)
    for k in ("dx", "poses", "disps"):
        np.testing.assert_array_equal(got[k], ref1[k], err_msg=k)   # bitwise: the BA is deterministic


def test_chol_stale_sync_area_after_an_aborted_solve_is_detected(ab_backends):
    """the entry check used to catch only the counters of a launch
    that ran to completion; an aborted launch leaves its ticket counter
    anywhere.  With the per-launch epoch the solve after an abort, launched on
    its unzeroed sync area, must still report status bit 2."""
    droid_backends = ab_backends   # the fault-injection hook ships in the testing builds only
    prob = synthetic.ba_problem("C3", H=16, W=24, seed=13)
    args = lambda p, d: (p, d, dev(prob["intrinsics"]), dev(prob["disps_sens"]), dev(prob["targets"]),
                         dev(prob["weights"]), dev(prob["eta"]), dev(prob["ii"]), dev(prob["jj"]), prob["t0"],
                         prob["t1"], 1, 1e-4, 0.1, False)
    poses, disps = dev(prob["poses"]), dev(prob["disps"])
    try:
        droid_backends.chol_set_fault_inject(droid_backends.CHOL_INJECT_ONCE)
        with pytest.raises(RuntimeError, match="timed out"):
            droid_backends.ba(*args(poses, disps))
        droid_backends.chol_set_fault_inject(droid_backends.CHOL_INJECT_STALE)
        with pytest.raises(RuntimeError, match="state corrupt"):
            droid_backends.ba(*args(poses, disps))
    finally:
        droid_backends.chol_set_fault_inject(droid_backends.CHOL_INJECT_OFF)
    np.testing.assert_array_equal(host(poses), prob["poses"])
    np.testing.assert_array_equal(host(disps), prob["disps"])
    got = _gpu_ba(prob, 1, 1e-4, 0.1, ab_backends)          # and the next solve on the same plan is clean
    assert np.isfinite(got["dx"]).all()


def _torchrun(nproc, args, timeout):
    env = dict(os.environ, PYTHONUNBUFFERED="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        os.path.join(HERE, "sharded_ba_worker.py")] + [str(a) for a in args],
                       env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=timeout)
    assert r.returncode == 0, r.stdout.decode(errors="replace")[-3000:]


@pytest.mark.timeout(300)
def test_ba_sharded_fault_on_one_rank_is_agreed(tmp_path):
    """the sharded BA all-reduces (MAX) the status words before each
    step is applied.  Rank 0 alone aborts its solves; both ranks must skip the
    same steps (poses and disparities bitwise equal across ranks, and unchanged
    when every step aborted) and both must raise."""
    prob = synthetic.ba_problem("C5", H=C5_HW[0], W=C5_HW[1])
    out = str(tmp_path / "inj")
    _torchrun(2, [out, C5_HW[0], C5_HW[1], "inject"], 280)
    d = [np.load(out + ".rank%d.npz" % r) for r in range(2)]
    for r in range(2):
        assert bool(d[r]["all_raised"]) and bool(d[r]["once_raised"]), "rank %d did not raise" % r
        # every GN step of the first call was skipped on every rank: nothing moved
        np.testing.assert_array_equal(d[r]["all_poses"], prob["poses"])
        np.testing.assert_array_equal(d[r]["all_disps"], prob["disps"])
    # the second call skipped its first step everywhere and applied the second
    # (identical all-reduced system -> identical solve on both ranks)
    np.testing.assert_array_equal(d[0]["once_poses"], d[1]["once_poses"])
    assert np.abs(d[0]["once_poses"] - prob["poses"]).max() > 0


@pytest.mark.timeout(480)
def test_ba_sharded_four_ranks_full_resolution(tmp_path):
    """the edge-sharded C5 BA at the config's 48x64 depth
    maps over 4 ranks (two middle ranks with both neighbours), every rank on
    cuda:0 over gloo, against the fp64 oracle at 1e-4.  The oracle runs while
    the ranks do."""
    prob = synthetic.ba_problem("C5", H=48, W=64)
    out = str(tmp_path / "c5full")
    env = dict(os.environ, PYTHONUNBUFFERED="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    proc = subprocess.Popen([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
                             "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                             os.path.join(HERE, "sharded_ba_worker.py"), out, "48", "64"],
                            env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    try:
        ref = oba.ba(**{k: prob[k] for k in KEYS}, iterations=2, lm=1e-5, ep=1e-2, motion_only=False)
        log, _ = proc.communicate(timeout=300)
    finally:
        if proc.poll() is None:
            proc.kill()
            proc.communicate()
    assert proc.returncode == 0, log.decode(errors="replace")[-3000:]
    covered = np.zeros(2048, bool)
    edges = 0
    for rank in range(4):
        d = np.load(out + ".rank%d.npz" % rank)
        lo, hi = (int(x) for x in d["own"])
        assert (0 < lo and hi < 2048) == (rank in (1, 2))
        edges += int(d["edges"])
        np.testing.assert_allclose(d["dx"], ref["dx"], atol=TOL, rtol=0)
        np.testing.assert_allclose(d["poses"], ref["poses"], atol=TOL, rtol=0)
        np.testing.assert_allclose(d["disps"][lo:hi], ref["disps"][lo:hi], atol=TOL, rtol=0)
        covered[lo:hi] = True
    assert covered.all() and edges == len(prob["ii"])
    assert np.abs(ref["dx"]).max() > 1e-4
