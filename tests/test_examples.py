"""The configs[0] harness (examples/image_dataloading.py): its host-side
plumbing on CPU, and one small GPU run through the decode path."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "examples"))


def test_source_split_and_batches(tmp_path):
    import image_dataloading as ex

    flist = tmp_path / "f.txt"
    flist.write_text("a\nb\n\nc\nd\ne\n")
    assert list(ex.source(str(flist), "/p/", 2, 0)) == ["/p/a", "/p/d"]  # line 2 is blank
    assert list(ex.source(str(flist), "", 2, 1)) == ["b", "c", "e"]
    assert list(ex.batches(iter(range(5)), 2)) == [[0, 1], [2, 3], [4]]


@pytest.mark.gpu
def test_synthetic_run_one_gpu():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "image_dataloading.py"),
                        "--synthetic", "96", "--batch-size", "16", "--num-threads", "2"],
                       capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["frames"] == 96 and rec["batches"] == 6 and rec["images_per_sec"] > 0
