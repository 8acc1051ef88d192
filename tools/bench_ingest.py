#!/usr/bin/env python3
"""Ground-truth ingestion throughput (§8f row 4): batches of B pointcloud_1024.npy
files to HBM.  Reference path: per-sample np.load (utils/datasets_old.py:37-38),
default collate (torch.stack), .cuda() (train.py:152-156).  This path:
GTPrefetcher (threaded native reader into pinned buffers, one async copy per
batch on a side stream).  Files live in a temp dir (page cache warm after the
first epoch, as in training)."""
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-pointcloudreconstruction_amd", "utils"))
import gt_ingest  # noqa: E402


def main():
    B, NB, N = 32, 40, 1024
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as d:
        paths = []
        for i in range(B * NB):
            p = os.path.join(d, f"m{i:05d}", "pointcloud_1024.npy")
            os.makedirs(os.path.dirname(p))
            np.save(p, rng.random((N, 3), dtype=np.float32))
            paths.append(p)
        batches = [paths[k * B:(k + 1) * B] for k in range(NB)]
        # warm the page cache once (training reads every file every epoch)
        for p in paths:
            np.load(p)

        def ref_epoch():
            out = None
            for bp in batches:
                out = torch.stack([torch.from_numpy(np.load(p)) for p in bp]).cuda()
            torch.cuda.synchronize()
            return out

        def pcm_epoch():
            out = None
            for g in gt_ingest.GTPrefetcher(batches, dev, N):
                out = g
            torch.cuda.synchronize()
            return out

        res = {}
        for name, fn in (("reference_np_load_stack_cuda", ref_epoch), ("gt_prefetcher", pcm_epoch)):
            fn()
            t0 = time.perf_counter()
            for _ in range(3):
                fn()
            dt = (time.perf_counter() - t0) / 3
            res[name] = {"ms_per_batch": dt * 1e3 / NB, "clouds_per_s": B * NB / dt,
                         "MB_per_s": B * NB * N * 12 / dt / 1e6}
        a, b = ref_epoch(), pcm_epoch()
        res["last_batch_equal"] = bool(torch.equal(a, b))
        res["config"] = f"{NB} batches x B={B} files of (1024,3) float32, warm page cache, threads={gt_ingest.default_threads()}"
        res["speedup"] = res["gt_prefetcher"]["clouds_per_s"] / res["reference_np_load_stack_cuda"]["clouds_per_s"]
        print(json.dumps(res))


if __name__ == "__main__":
    main()
