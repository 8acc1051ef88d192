"""Config-4 training-step benchmark (BASELINE.json configs[3]).

    python tools/bench_train.py [--batch 16] [--steps 10] [--warmup 3] [--epoch 1]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 ... tools/bench_train.py ...

One step = generator forward on a synthetic [B,3,128,128] batch, Chamfer +
EMD (eps 0.05, 3000 iterations: loss/loss.py:23) against [B,1024,3] clouds,
backward, fused Adam; DDP over RCCL when launched with several ranks (weak
scaling: --batch per rank; the reference's 128 over 8 GPUs is 16 per rank).
Random-init weights (seeded_init) and synthetic data: the checkpoint and
ShapeNet are absent.  Phase times come from HIP events on the step's stream;
the loss-path share is also measured standalone (loss forward + backward on
the same predicted clouds).  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "train"))
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "metric"))
import train_step as T  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16, help="clouds per rank")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--epoch", type=int, default=1, help="1..30: CD+EMD loss, 31..50: EMD only")
    ap.add_argument("--emd-iters", type=int, default=3000)
    ap.add_argument("--emd-eps", type=float, default=0.05)
    ap.add_argument("--bucket-mb", type=float, default=100.0)
    ap.add_argument("--channels-last", action="store_true", help="NHWC activations for the encoder")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL); gloo only to rehearse several ranks on one GPU")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)
    torch.backends.cudnn.benchmark = True  # train.py:85

    step = T.TrainStep(device=dev, emd_eps=args.emd_eps, emd_iters=args.emd_iters,
                       bucket_cap_mb=args.bucket_mb, seed=0,
                       channels_last=args.channels_last)
    step.set_epoch(args.epoch)
    images, points = T.synthetic_batch(args.batch, 1024, dev, seed=rank)

    for _ in range(args.warmup):
        step(images, points, args.epoch)
    torch.cuda.synchronize()

    # phase split of one step (events on the current stream; no host sync inside)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
    ev[0].record()
    _, _, fake = step.gen(images.contiguous(memory_format=torch.channels_last) if args.channels_last else images)
    ev[1].record()
    pred = fake.transpose(2, 1)
    w = T.loss_weights(args.epoch, step.lambda_cd, step.lambda_emd)
    cd = step.loss_fn.get_chamfer_loss(pred, points)
    emd = step.loss_fn.get_emd_loss(pred, points, eps=args.emd_eps, iters=args.emd_iters)
    total = emd * w[1] if w[0] == 0.0 else cd * w[0] + emd * w[1]
    ev[2].record()
    step.opt.zero_grad(set_to_none=True)
    total.backward()
    ev[3].record()
    step.opt.step()
    ev[4].record()
    torch.cuda.synchronize()
    phases = {k: ev[i].elapsed_time(ev[i + 1]) for i, k in
              enumerate(["generator_fwd_ms", "loss_fwd_ms", "backward_ms", "adam_ms"])}

    # standalone loss path on the same predicted clouds: forward + backward
    leaf = pred.detach().contiguous().requires_grad_(True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 3
    e0.record()
    for _ in range(reps):
        c = step.loss_fn.get_chamfer_loss(leaf, points)
        m = step.loss_fn.get_emd_loss(leaf, points, eps=args.emd_eps, iters=args.emd_iters)
        (c * w[0] + m * w[1]).backward()
    e1.record()
    torch.cuda.synchronize()
    loss_ms = e0.elapsed_time(e1) / reps

    # per-step record: each step trains the generator, so the next step's
    # predictions -- and the EMD auction's work on them -- differ.  Events
    # time every step (no host sync); a forward hook keeps each step's
    # predicted clouds (one small copy) so the auction's iterations and bids
    # per step are counted afterwards, outside the timed region.
    caps = []
    hook = step.gen.register_forward_hook(
        lambda m, i, o: caps.append(o[2].detach().transpose(2, 1).contiguous()))
    sev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sev[0].record()
    for i in range(args.steps):
        logged = step(images, points, args.epoch)
        sev[i + 1].record()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    hook.remove()
    step_ms = [sev[i].elapsed_time(sev[i + 1]) for i in range(args.steps)]
    emd_work = []
    import pcm_hip
    b, n = points.shape[0], points.shape[1]
    for pred_i in caps:
        st = torch.zeros(3 * args.emd_iters + 16 + b, dtype=torch.int32, device=dev)
        d = torch.empty(b, n, device=dev)
        a_ = torch.empty(b, n, dtype=torch.int32, device=dev)
        pcm_hip.emd_forward(pred_i, points.contiguous(), args.emd_eps, args.emd_iters, d, a_, stats=st, diag=1)
        e0.record()
        pcm_hip.emd_forward(pred_i, points.contiguous(), args.emd_eps, args.emd_iters, d, a_)
        e1.record()
        torch.cuda.synchronize()
        h = st.cpu()[:2 * args.emd_iters].view(-1, 2)
        # elements whose master timed out on a helper job and scanned the items
        # itself (exact, but a silent fall back to master-only scans)
        timeouts = pcm_hip.emd_timeouts(pcm_hip.emd_workspace(dev, b, n), b, n)
        emd_work.append({"iterations_with_bidders": int((h[:, 0] > 0).sum()), "bids": int(h[:, 0].sum()),
                         "full_scans": int(h[:, 1].sum()), "emd_fwd_ms": e0.elapsed_time(e1),
                         "helper_timeouts": timeouts})
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms = dt * 1e3 / args.steps
    vals = logged.tolist()
    if rank == 0:
        print(json.dumps({
            "metric": "3D-FENet training step (config 4)", "value": args.batch * world / (ms / 1e3),
            "unit": "samples/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms, "higher_is_better": True, "scaling": "weak", "dtype": "f32",
            "data": "synthetic images [B,3,128,128] in [-1,1], GT clouds rand [0,1); seeded random-init generator",
            "config": {"workload": "train.py step: generator fwd, Chamfer+EMD loss, backward, Adam",
                       "batch_per_gpu": args.batch, "global_batch": args.batch * world, "epoch": args.epoch,
                       "emd_eps": args.emd_eps, "emd_iters": args.emd_iters, "params": 177276968,
                       "parallelism": f"ddp{world}" + ("" if args.dist_backend == "nccl" else f" ({args.dist_backend})"),
                       "bucket_cap_mb": args.bucket_mb,
                       "channels_last": args.channels_last},
            "phases_ms": phases, "loss_path_ms": loss_ms, "loss_path_share": loss_ms / ms,
            "per_step": [dict(step_ms=t, **w_) for t, w_ in zip(step_ms, emd_work)],
            "last_losses": {"total": vals[0], "chamfer": vals[1], "emd": vals[2]},
        }))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
