"""Ground-truth cloud ingestion -- SURVEY.md §8f row 4.

Reference: ``GetShapenetDataset.__getitem__`` (utils/datasets_old.py:29-52) builds
``data_dir_pcl + modelnames[index] + '/pointcloud_' + str(numpoints) + '.npy'``
and ``np.load``s it for every sample; the DataLoader collates the batch and
train.py moves it to the GPU with ``.cuda()`` (train.py:152-156).

Here the ground-truth half of that path is batched:
  ShapenetGTIndex      the reference's sample index -> file mapping (24 views
                       per model, utils/datasets_old.py:6 and :23-27)
  load_gt_batch        one libpcm call reads a whole batch of .npy files with a
                       thread pool into one (pinned) [B, npoints, 3] float32
                       buffer -- values == np.load(path).astype(float32)
  GTPrefetcher         iterator: batch k+1 is read on a background thread into
                       the other pinned buffer while batch k is in use, and
                       each batch reaches HBM in ONE non-blocking copy on a side
                       stream that the consumer's stream waits on (no host sync)

The file reader is native (csrc/npy_ingest.cpp, in libpcm_hip.so); there is no
numpy fallback.
"""
import ctypes
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import torch

_METRIC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "metric")
if _METRIC not in sys.path:
    sys.path.append(_METRIC)
import pcm_hip  # noqa: E402

NUM_VIEWS = 24  # utils/datasets_old.py:6


def _lib():
    L = pcm_hip.load_library()
    if not getattr(L, "_pcm_ingest_bound", False):
        L.pcm_npy_cloud_points.restype = ctypes.c_int
        L.pcm_npy_cloud_points.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]
        L.pcm_npy_load_clouds.restype = ctypes.c_int
        L.pcm_npy_load_clouds.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.c_int, ctypes.c_int,
                                          ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L._pcm_ingest_bound = True
    return L


def cloud_points(path) -> int:
    """Row count of an (N, 3) float .npy cloud."""
    n = ctypes.c_int(0)
    rc = _lib().pcm_npy_cloud_points(os.fsencode(path), ctypes.byref(n))
    if rc != 0:
        raise pcm_hip.PcmError(f"{path}: {pcm_hip.strerror(rc)} (status {rc})")
    return n.value


def default_threads() -> int:
    return max(1, min(16, os.cpu_count() or 1))


def load_gt_batch(paths, npoints=1024, out=None, nthreads=None, pin=None):
    """Read len(paths) clouds of shape (npoints, 3) into a float32 tensor
    [B, npoints, 3] (``out`` if given, else new; pinned when a GPU is
    visible unless pin=False).  Raises PcmError naming the first bad file."""
    paths = [os.fsencode(p) for p in paths]
    b = len(paths)
    if out is None:
        if pin is None:
            pin = torch.cuda.is_available()
        out = torch.empty((b, npoints, 3), dtype=torch.float32, pin_memory=bool(pin))
    if out.dtype != torch.float32 or out.device.type != "cpu" or not out.is_contiguous():
        raise ValueError("out must be a contiguous float32 host tensor")
    if out.shape[0] < b or tuple(out.shape[1:]) != (npoints, 3):
        raise ValueError(f"out must hold [{b}, {npoints}, 3] (got {tuple(out.shape)})")
    arr = (ctypes.c_char_p * max(b, 1))(*paths)
    bad = ctypes.c_int(-1)
    rc = _lib().pcm_npy_load_clouds(arr, b, int(npoints), ctypes.c_void_p(out.data_ptr()),
                                    int(nthreads or default_threads()), ctypes.byref(bad))
    if rc != 0:
        where = os.fsdecode(paths[bad.value]) if 0 <= bad.value < b else "?"
        raise pcm_hip.PcmError(f"{where}: {pcm_hip.strerror(rc)} (status {rc})")
    return out[:b]


class ShapenetGTIndex:
    """The reference dataset's sample -> ground-truth file mapping
    (GetShapenetDataset.__init__ / __getitem__, utils/datasets_old.py:13-38):
    every model of every category contributes NUM_VIEWS consecutive samples."""

    def __init__(self, data_dir_pcl, models, cats, numpoints=1024):
        self.data_dir_pcl = data_dir_pcl
        self.numpoints = numpoints
        self.modelnames = []
        for cat in cats:
            for filename in models[cat]:
                for _ in range(NUM_VIEWS):
                    self.modelnames.append(filename)

    def __len__(self):
        return len(self.modelnames)

    def path(self, index):
        return self.data_dir_pcl + self.modelnames[index] + '/pointcloud_' + str(self.numpoints) + '.npy'

    def batch_paths(self, indices):
        return [self.path(int(i)) for i in indices]


class GTPrefetcher:
    """Iterate device batches [B, npoints, 3] float32 for a sequence of path
    lists.  Reading batch k+1 (thread pool, pinned buffer k+1 mod 2) overlaps
    the consumer's work on batch k; the copy to HBM is one non_blocking copy on
    a side stream, and the consumer's current stream waits on it."""

    def __init__(self, path_batches, device, npoints=1024, nthreads=None):
        self.batches = [list(p) for p in path_batches]
        self.device = torch.device(device)
        self.npoints = npoints
        self.nthreads = nthreads or default_threads()
        bmax = max((len(p) for p in self.batches), default=0)
        self.host = [torch.empty((bmax, npoints, 3), dtype=torch.float32, pin_memory=True) for _ in range(2)]
        self.copied = [None, None]  # event: the last H2D copy out of host[j] finished
        self.stream = torch.cuda.Stream(self.device)

    def __len__(self):
        return len(self.batches)

    def _read(self, k):
        j = k % 2
        if self.copied[j] is not None:
            self.copied[j].synchronize()  # host[j] may still be feeding batch k-2's copy
        load_gt_batch(self.batches[k], self.npoints, out=self.host[j], nthreads=self.nthreads)

    def __iter__(self):
        n = len(self.batches)
        if n == 0:
            return
        with ThreadPoolExecutor(max_workers=1) as ex:  # one long-lived reader thread
            fut = ex.submit(self._read, 0)
            for k in range(n):
                fut.result()  # re-raises the reader's PcmError
                j = k % 2
                b = len(self.batches[k])
                consumer = torch.cuda.current_stream(self.device)
                self.stream.wait_stream(consumer)  # device memory reuse order
                with torch.cuda.stream(self.stream):
                    d = self.host[j][:b].to(self.device, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self.stream)
                self.copied[j] = ev
                consumer.wait_stream(self.stream)
                d.record_stream(consumer)
                if k + 1 < n:  # read the next batch while the consumer works on this one
                    fut = ex.submit(self._read, k + 1)
                yield d
