"""The Lego checkpoint: the weights-only reader of the reference's
original-NeRF .npy object arrays, and the distilled NeRFModel-layout checkpoint."""
import hashlib
import json
import os
import pickle
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))

from lego.npy_static import RefusedPickle, parse_pickle, read_object_npy  # noqa: E402
from nerf_amd import weights as W  # noqa: E402

LEGO_DIR = "/root/reference/data/lego_example_weights"
GOLDEN = os.path.join(REPO, "tests", "golden")


def _obj_npy(path, arrays):
    obj = np.empty(len(arrays), dtype=object)
    for i, a in enumerate(arrays):
        obj[i] = a
    np.save(path, obj, allow_pickle=True)       # writing only: the reader below unpickles nothing


@pytest.mark.parametrize("protocol_dtype", ["<f4", "<f8", "<i4", ">f4"])
def test_reader_roundtrips_object_arrays(tmp_path, protocol_dtype):
    rng = np.random.RandomState(0)
    arrays = [rng.randn(7, 5).astype(protocol_dtype), rng.randn(3).astype(protocol_dtype),
              np.asfortranarray(rng.randn(4, 6)).astype(protocol_dtype), np.zeros((0, 3), protocol_dtype)]
    p = str(tmp_path / "w.npy")
    _obj_npy(p, arrays)
    got = read_object_npy(p)
    assert len(got) == len(arrays)
    for a, b in zip(arrays, got):
        assert a.shape == b.shape and np.array_equal(a, b) and b.dtype == a.dtype.newbyteorder("=")


class _Evil:
    def __reduce__(self):
        return (os.system, ("echo should-never-run",))


@pytest.mark.parametrize("payload", [
    lambda: pickle.dumps(_Evil(), protocol=2),                          # GLOBAL posix system + REDUCE
    lambda: pickle.dumps(_Evil(), protocol=4),                          # STACK_GLOBAL form
    lambda: pickle.dumps({"a": 1}, protocol=2),                         # EMPTY_DICT: not in the subset
    lambda: pickle.dumps(np.float64(1.5), protocol=2),                  # numpy scalar global
    lambda: b"\x80\x02cbuiltins\neval\nq\x00X\x03\x00\x00\x001+1q\x01\x85q\x02Rq\x03.",
])
def test_reader_refuses_other_globals_and_opcodes(payload):
    with pytest.raises(RefusedPickle):
        parse_pickle(payload())


def test_reader_refuses_a_non_object_npy(tmp_path):
    p = str(tmp_path / "plain.npy")
    np.save(p, np.ones(3, np.float32))
    with pytest.raises(RefusedPickle):
        read_object_npy(p)


@pytest.mark.skipif(not os.path.isdir(LEGO_DIR), reason="the reference checkout (build container only)")
def test_reader_reads_the_reference_lego_weights():
    ref = json.load(open(os.path.join(GOLDEN, "lego_teacher_arrays.json")))
    for name in ("model_200000", "model_fine_200000"):
        arrs = read_object_npy(os.path.join(LEGO_DIR, name + ".npy"))
        assert [list(a.shape) for a in arrs] == ref[name]["shapes"]
        assert [hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16] for a in arrs] == ref[name]["sha256"]
        assert all(a.dtype == np.float32 and np.isfinite(a).all() for a in arrs)


@pytest.mark.skipif(not os.path.exists(W.LEGO_NPZ), reason="distilled checkpoint not built yet")
def test_distilled_lego_checkpoint_layout(tmp_path):
    coarse, fine = W.lego_models()
    meta = json.load(open(W.LEGO_NPZ.replace(".npz", ".json")))
    assert W.state_dict_digest(coarse) == meta["coarse_digest"]
    assert W.state_dict_digest(fine) == meta["fine_digest"]
    p = W.write_lego_checkpoint(str(tmp_path / "lego.pth"))
    c2, f2 = W.load_checkpoint(p)
    assert W.state_dict_digest(f2) == meta["fine_digest"] and W.state_dict_digest(c2) == meta["coarse_digest"]
    c3, f3 = W.load_checkpoint(W.LEGO_NPZ)
    assert W.state_dict_digest(f3) == meta["fine_digest"]
    # the distillation's own held-out report
    assert meta["report"]["fine"]["psnr_db_mean"] > 20.0
