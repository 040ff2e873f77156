"""Every BASELINE.json config inside `pytest -m gpu` (one GPU box):

* configs[0]: examples/image_dataloading.py on 1,000 local JPEG files, one
  decoded image of every batch checked against the oracle;
* configs[2]: bench.py's 8-rank launch (2048 -> 8 x 256) rehearsed on one
  GPU: 8 ranks, disjoint contiguous slices, every rank's oracle check;
* configs[4]: bench_stream.py's N-rank tar stream rehearsed on one GPU,
  each rank's first batch of the last timed pass checked against the oracle.

The multi-GPU *rates* are the driver's 8-GPU run; these tests pin the launch
paths and pixels of the same commands on one device.
"""

import glob
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PAD224 = dict(fit_w=224, fit_h=224, aspect="decrease", pad_w=224, pad_h=224)

pytestmark = pytest.mark.gpu


def _run(args, timeout):
    r = subprocess.run([sys.executable, *args], capture_output=True, text=True, timeout=timeout,
                       cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_configs0_dataloading_1k_files_pixels(oracle, tmp_path):
    out = str(tmp_path / "samples")
    rec = _run([os.path.join(ROOT, "examples", "image_dataloading.py"), "--synthetic", "1000",
                "--batch-size", "32", "--num-threads", "4", "--sample-out", out], 240)
    assert rec["frames"] == 1000 and rec["batches"] == 32
    z = np.load(out + ".w0.npz")
    ks = sorted(int(k[4:]) for k in z.files if k.startswith("rgb_"))
    assert len(ks) == 32  # one sample per batch
    rs = oracle.Resize(**PAD224)
    for k in ks:
        ref = oracle.decode_resize(z[f"jpeg_{k}"].tobytes(), rs, "rgb24")
        np.testing.assert_array_equal(z[f"rgb_{k}"], ref, strict=True)


def test_configs2_eight_rank_launch_rehearsed(tmp_path):
    rec = _run(["bench.py", "--gpus", "8", "--batch", "256", "--rehearse-one-gpu", "--steps", "3",
                "--warmup", "1", "--lanes1-steps", "0", "--no-cpu-baseline", "--bind", "split"], 600)
    assert rec["n_gpus"] == 8 and rec["config"]["global_batch"] == 2048
    ranks = sorted(rec["ranks"], key=lambda r: r["rank"])
    assert [r["rank"] for r in ranks] == list(range(8))
    slices = [tuple(r["slice"]) for r in ranks]
    assert slices == [(256 * i, 256 * (i + 1)) for i in range(8)]  # disjoint, covering
    for r in ranks:
        assert r["oracle_check"].endswith("bit-exact vs oracle"), r
        assert r["images_per_sec"] > 0
    _assert_disjoint_cores(ranks)


def _assert_disjoint_cores(ranks):
    """Each rank bound itself to its own cores of its GPU's NUMA node
    (spdl_amd.distributed.bind_rank_cpus), the sets pairwise disjoint when
    the box has a core per rank."""
    assert all(r["bind"] == "split" for r in ranks), ranks
    sets = [set(r["cpus"]) for r in ranks]
    assert all(sets), ranks
    if sum(len(s) for s in sets) >= len(sets) and len(set().union(*sets)) >= len(sets):
        for i in range(len(sets)):
            for j in range(i + 1, len(sets)):
                assert not (sets[i] & sets[j]), (i, j, sets)


def test_configs4_stream_ranks_rehearsed(oracle, tmp_path):
    from spdl_amd.synthetic import synthetic_batch

    out = str(tmp_path / "stream")
    rec = _run(["bench_stream.py", "--gpus", "2", "--rehearse-one-gpu", "--images", "512",
                "--passes", "2", "--sample-out", out, "--sample-images", "16"], 600)
    assert rec["n_gpus"] == 2 and len(rec["ranks"]) == 2
    datas = synthetic_batch(512, distinct=32)
    rs = oracle.Resize(**PAD224)
    files = sorted(glob.glob(out + ".r*.npz"))
    assert len(files) == 2
    for f in files:
        z = np.load(f)
        for name, rgb in zip(z["names"], z["rgb"]):
            i = int(str(name).rsplit("/", 1)[1][:-4])
            np.testing.assert_array_equal(rgb, oracle.decode_resize(datas[i], rs, "rgb24"),
                                          strict=True)


def test_configs4_stream_eight_ranks_rehearsed(oracle, tmp_path):
    """configs[4] as the driver would launch it on an 8-GPU node (8 stream
    ranks, each its own shard of the tar stream, pinned ring, copy pool sized
    for LOCAL_WORLD_SIZE=8), rehearsed on one GPU; every rank's samples of
    its last timed pass checked against the oracle."""
    from spdl_amd.synthetic import synthetic_batch

    out = str(tmp_path / "stream8")
    rec = _run(["bench_stream.py", "--gpus", "8", "--rehearse-one-gpu", "--images", "512",
                "--passes", "1", "--warmup-passes", "1", "--sample-out", out,
                "--sample-images", "8", "--bind", "split"], 900)
    assert rec["n_gpus"] == 8 and len(rec["ranks"]) == 8
    _assert_disjoint_cores(rec["ranks"])
    datas = synthetic_batch(512, distinct=32)
    rs = oracle.Resize(**PAD224)
    refs = {}
    files = sorted(glob.glob(out + ".r*.npz"))
    assert len(files) == 8
    for f in files:
        z = np.load(f)
        assert len(z["names"]) > 0
        for name, rgb in zip(z["names"], z["rgb"]):
            i = int(str(name).rsplit("/", 1)[1][:-4])
            if i not in refs:
                refs[i] = oracle.decode_resize(datas[i], rs, "rgb24")
            np.testing.assert_array_equal(rgb, refs[i], strict=True)
