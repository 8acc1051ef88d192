"""Ground-truth ingestion (§8f row 4): the native .npy batch reader against
np.load (the reference's reader, utils/datasets_old.py:37-38), the reference's
index -> path mapping, and (GPU) the prefetching copy path."""
import os

import numpy as np
import pytest
import torch

import gt_ingest
import pcm_hip


def _write(path, arr, version=None):
    if version is None:
        np.save(path, arr)
    else:
        with open(path, "wb") as f:
            np.lib.format.write_array(f, arr, version=version)
    return path


@pytest.fixture()
def clouds(tmp_path):
    rng = np.random.default_rng(0)
    files, refs = [], []
    variants = [
        ("f4", lambda a: a.astype("<f4"), None),
        ("f8", lambda a: a.astype("<f8"), None),
        ("be4", lambda a: a.astype(">f4"), None),
        ("be8", lambda a: a.astype(">f8"), None),
        ("fortran", lambda a: np.asfortranarray(a.astype("<f4")), None),
        ("v2", lambda a: a.astype("<f4"), (2, 0)),
        ("v3", lambda a: a.astype("<f8"), (3, 0)),
    ]
    for k, (name, cast, ver) in enumerate(variants * 3):
        a = cast(rng.standard_normal((1024, 3)) * (10.0 ** (k % 5 - 2)))
        p = _write(str(tmp_path / f"{name}_{k}.npy"), a, ver)
        files.append(p)
        refs.append(np.load(p).astype(np.float32))
    return files, np.stack(refs)


def test_batch_matches_np_load(clouds):
    files, ref = clouds
    for nthreads in (1, 3, 16):
        out = gt_ingest.load_gt_batch(files, 1024, nthreads=nthreads, pin=False)
        assert out.dtype == torch.float32 and tuple(out.shape) == (len(files), 1024, 3)
        np.testing.assert_array_equal(out.numpy(), ref)


def test_float64_rounding_matches_numpy(tmp_path):
    # values that round differently under truncation vs round-to-nearest-even
    a = np.array([[1.0 + 2.0 ** -24, 1.0 + 3 * 2.0 ** -24, -1.0 - 2.0 ** -24],
                  [1e-45, 3.4028235e38, -0.0]] * 2, dtype=np.float64)
    p = _write(str(tmp_path / "r.npy"), a)
    out = gt_ingest.load_gt_batch([p], a.shape[0], pin=False)
    np.testing.assert_array_equal(out[0].numpy().view(np.uint32), a.astype(np.float32).view(np.uint32))


def test_cloud_points_and_out_buffer(clouds):
    files, ref = clouds
    assert gt_ingest.cloud_points(files[0]) == 1024
    buf = torch.empty(32, 1024, 3)
    got = gt_ingest.load_gt_batch(files[:5], 1024, out=buf)
    assert got.data_ptr() == buf.data_ptr() and got.shape[0] == 5
    np.testing.assert_array_equal(got.numpy(), ref[:5])


@pytest.mark.parametrize("kind", ["missing", "shape", "npoints", "truncated", "not_npy", "int_dtype", "3d"])
def test_errors_name_the_file(tmp_path, clouds, kind):
    files, _ = clouds
    bad = str(tmp_path / f"bad_{kind}.npy")
    if kind == "shape":
        np.save(bad, np.zeros((1024, 4), np.float32))
    elif kind == "npoints":
        np.save(bad, np.zeros((2048, 3), np.float32))
    elif kind == "truncated":
        np.save(bad, np.zeros((1024, 3), np.float32))
        with open(bad, "r+b") as f:
            f.truncate(os.path.getsize(bad) - 5)
    elif kind == "not_npy":
        with open(bad, "wb") as f:
            f.write(b"definitely not a numpy file" * 10)
    elif kind == "int_dtype":
        np.save(bad, np.zeros((1024, 3), np.int32))
    elif kind == "3d":
        np.save(bad, np.zeros((1024, 3, 1), np.float32))
    batch = files[:3] + [bad] + files[3:6]
    with pytest.raises(pcm_hip.PcmError, match=os.path.basename(bad)):
        gt_ingest.load_gt_batch(batch, 1024, pin=False, nthreads=4)


def test_shapenet_index_matches_reference_layout():
    models = {"02691156": ["02691156/a1", "02691156/b2"], "03001627": ["03001627/c3"]}
    idx = gt_ingest.ShapenetGTIndex("/data/pcl/", models, ["02691156", "03001627"], numpoints=1024)
    assert len(idx) == 3 * 24
    # utils/datasets_old.py:37: data_dir_pcl + modelnames[index] + '/pointcloud_' + str(numpoints) + '.npy'
    assert idx.path(0) == "/data/pcl/02691156/a1/pointcloud_1024.npy"
    assert idx.path(23) == "/data/pcl/02691156/a1/pointcloud_1024.npy"
    assert idx.path(24) == "/data/pcl/02691156/b2/pointcloud_1024.npy"
    assert idx.path(71) == "/data/pcl/03001627/c3/pointcloud_1024.npy"
    assert idx.batch_paths([0, 48]) == [idx.path(0), idx.path(48)]


@pytest.mark.gpu
def test_prefetcher_delivers_batches_on_device(clouds, cuda):
    files, ref = clouds
    batches = [files[i:i + 4] for i in range(0, len(files), 4)]
    out = []
    for d in gt_ingest.GTPrefetcher(batches, cuda, 1024, nthreads=4):
        assert d.device.type == "cuda" and d.dtype == torch.float32
        out.append((d * 1.0).cpu().numpy())  # consumer work on the current stream
    np.testing.assert_array_equal(np.concatenate(out), ref)


@pytest.mark.gpu
def test_prefetcher_feeds_the_loss(clouds, cuda):
    """GT batch straight into the one-launch Chamfer loss."""
    import dist_chamfer_3D
    files, ref = clouds
    batches = [files[0:4], files[4:8]]
    pred = torch.rand(4, 1024, 3, device=cuda)
    for k, gt in enumerate(gt_ingest.GTPrefetcher(batches, cuda, 1024)):
        loss = dist_chamfer_3D.chamfer_3DLoss()(pred, gt)
        d1, d2, _, _ = dist_chamfer_3D.chamfer_3DDist()(pred, torch.from_numpy(ref[4 * k:4 * k + 4]).to(cuda))
        torch.testing.assert_close(loss, d1.mean() + d2.mean(), rtol=1e-5, atol=1e-6)
