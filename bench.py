#!/usr/bin/env python3
"""Benchmark of the Chamfer3D / EMD hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--eager] [--no-cpu]

One step = one pass of the hot path over one synthetic batch, exactly as a
training step of train.py:162-176 drives it: Chamfer3D forward (both
directions, B=32, N=M=1024 per GPU -- BASELINE config 2), the loss
mean(dist1)+mean(dist2) (loss/loss.py:36), the cross-rank RCCL all-reduce of
that scalar when N>1, and the Chamfer3D backward with graddist = 1/(B*N) (the
gradient torch's mean feeds it).  Inputs are resident in HBM before timing.
The step runs as ONE launch of pcm_chamfer_loss_grad (forward, loss and both
clouds' gradients; csrc/chamfer_filt.hip); --two-launch runs it as the fused-
loss forward + the backward kernel instead (both are reported).
The timed region replays a captured 20-step hipGraph of the step (the first
replay paid in warmup), at N=1 and at N>1 alike: N>1 only adds each step's
loss all-reduce to the same graph, so a 1->N curve isolates the collective.
Round 6's matched A/B against K direct launches from one C call
(pcm_chamfer_loss_grad_steps, --c-loop) gave 15.71 against 15.82 us per step
at the driver's K = 20 (tools/ab_launch_form.py,
profiles/r06/ab_launch_form_r06c.txt); --eager times the Python wrapper.  The
GPU-side time of the timed region (HIP events at its edges, on the kernel's
stream) is the dominant kernel's duration in `roofline`.
Order: the headline's W warmup steps and K timed steps first, then the legs
reported beside it (ICP, the unchanged caller's call sequence, config 5, EMD;
side_legs), then the CPU baseline.  --side-legs first runs those legs before
the warmup instead: not faster (same box, profiles/r05/bench_side_legs_r05o.txt).

value = point pairs evaluated per second over all ranks (2*B*N*M per rank per
step / max-over-ranks wall time).  EMD (BASELINE config 3: B=16, N=1024,
50 iterations, eps=0.005) is reported alongside as iterations/s, and the dense
fp16 Chamfer (BASELINE config 5: B=8, N=M=16384) as point-pairs/s.

Multi-GPU: one process per GPU, batches sharded (weak scaling: each rank owns
its own B=32 clouds).  `python bench.py --gpus N` with no WORLD_SIZE in the
environment relaunches itself as N ranks under torch.distributed.run (before
any GPU call) and exits with their status; under torchrun WORLD_SIZE must equal
--gpus.  At N>1 every step all-reduces ITS OWN loss vector over RCCL (the
north_star contract): the step's kernel and, on a side stream, the 12-byte
all-reduce of that step's losses are captured together into the hipGraph, so
step i's collective overlaps step i+1's kernel and the graph holds one
collective per step.  If the collective cannot be captured (gloo, or a capture
error) each step replays a one-step graph and all-reduces eagerly.  The
bucketed form (one all-reduce of GRAPH_STEPS steps' losses per replay) is
reported beside it.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "3d-pointcloudreconstruction_amd")
sys.path.insert(0, os.path.join(PKG, "metric"))
import pcm_hip  # noqa: E402

B, N, M = 32, 1024, 1024           # BASELINE config 2 (per GPU)
EMD_B, EMD_N, EMD_EPS, EMD_ITERS = 16, 1024, 0.005, 50   # BASELINE config 3
GRAPH_STEPS = 20                   # steps captured per hipGraph replay (the driver times 20)
BENCH_SEED = 1234                  # rank r's clouds: torch.Generator seed BENCH_SEED + r (tools/ab_chamfer.py too)
# the forward kernel instance the step launches at this size (csrc/chamfer.hip
# default_fwd_variant) and the committed rocprofv3 counter summary it is looked
# up in for roofline.traffic (tools/pmc_passes.sh + tools/pmc_summarize.py)
FWD_KERNEL = "chamfer_fwd_filt_kernel<float, 8, 4, 16, 1024, 3>"  # default fused-loss forward (clouds <= 1024)
BWD_KERNEL = "chamfer_bwd_slots_kernel"
FUSED_KERNEL = "chamfer_loss_grad_kernel<8, 4, 16, 1024, false, true, false, false, false, false, false, 0, 0, false>"  # default variant 7 (8-byte argmin granules, both clouds copied into LDS for the gradient phase)
# the newest committed counter summary (profiles/rNN/pmc_summary.json)
PMC_SUMMARY = next((p for p in (os.path.join(REPO, "profiles", r, "pmc_summary.json") for r in ("r06", "r05"))
                    if os.path.exists(p)), os.path.join(REPO, "profiles", "r05", "pmc_summary.json"))

# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md, chip-level parameters)
HBM_PEAK_GBS = 8000.0
FP32_VALU_PEAK_TFLOPS = 157.3
# VALU issue: a wave64 instruction every 2 cycles per SIMD (guide, per-instruction
# constants: v_fma_f32 2 cyc) = 32 lane-ops/cycle/SIMD x 4 SIMD x 256 CU x 2.4 GHz
VALU_LANE_OPS_PEAK = 256 * 4 * 32 * 2.4e9
# the reference's Bid (emd_cuda.cu:139-155) per (bidder, object) pair: 3 sub,
# 1 mul + 2 fma, sqrt, 2 f32->f64 cvt, 2 f64 sub, f64->f32 cvt, 2 compares
# + 3 selects of the top-2 update ~= 20 lane-ops
EMD_LANE_OPS_PER_PAIR = 20
# algorithmic FLOPs per point pair of the squared distance: 3 sub + 3 mul + 2 add
FLOP_PER_PAIR = 8
# algorithmic HBM bytes of the forward launch: read both clouds, write
# dist1/dist2 (f32) + idx1/idx2 (i32)  
FWD_BYTES = 2 * B * N * 12 + 4 * B * N * 4
BWD_BYTES = 2 * B * N * 12 + 2 * B * N * 4 + 2 * B * N * 4 + 2 * B * N * 12
# the one-launch loss + gradient: read both clouds, write dist + idx (both
# directions) and both gradients (the constant graddist is a kernel argument)
FUSED_BYTES = 2 * B * N * 12 + 4 * B * N * 4 + 2 * B * N * 12


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="ranks (one per GPU); default: WORLD_SIZE under torchrun, else 1")
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--eager", action="store_true", help="no hipGraph capture (Python wrapper per step)")
    p.add_argument("--graph", action="store_true",
                   help="(the default form; kept for old command lines)")
    p.add_argument("--c-loop", action="store_true",
                   help="N=1: time K direct launches from one C call (pcm_chamfer_loss_grad_steps) instead of "
                        "replays of the captured 20-step hipGraph (matched A/B: profiles/r06/ab_launch_form_r06c.txt)")
    p.add_argument("--two-launch", action="store_true",
                   help="step = fused-loss forward + backward kernel (not the one-launch loss+gradient)")
    p.add_argument("--tune-variant", type=int, default=None,
                   help="A/B only: the headline step runs this fused variant of the tuning build "
                        "(libpcm_hip_tune.so) instead of the product entry; marked in config")
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    p.add_argument("--side-legs", choices=("first", "last"), default="last",
                   help="run the legs reported beside the headline after its timed region (default) or before "
                        "its warmup (same box, r05o: 16.08/16.15 us per step first, 15.88/15.96 last)")
    p.add_argument("--no-emd", action="store_true", help="skip the EMD leg")
    p.add_argument("--no-dense", action="store_true", help="skip the dense fp16 (config 5) leg")
    p.add_argument("--no-icp", action="store_true", help="skip the ICP (evaluation alignment) leg")
    p.add_argument("--no-ref-call", action="store_true",
                   help="skip the leg that times loss/loss.py:34-36's literal call sequence")
    p.add_argument("--dist-backend", default="nccl",
                   help="torch.distributed backend for N>1 (nccl = RCCL; gloo only to rehearse "
                        "several ranks on one GPU)")
    p.add_argument("--force-dist", action="store_true",
                   help="run the N>1 code path (process group, per-step collective) even with one rank: "
                        "a single-GPU rehearsal of the RCCL capture")
    p.add_argument("--eager-allreduce", action="store_true",
                   help="N>1: all-reduce each step's loss eagerly instead of inside the graph")
    return p.parse_args(argv)


def resolve_launch(gpus, env):
    """How this invocation runs: ("self", world) -- run the benchmark in this
    process as one of `world` ranks -- or ("spawn", n) -- relaunch as n ranks
    under torch.distributed.run.  --gpus N with WORLD_SIZE unset spawns N ranks
    (N > 1); under a launcher WORLD_SIZE is authoritative and --gpus, when
    given, must equal it."""
    ws = env.get("WORLD_SIZE")
    if ws is None or ws == "":
        n = 1 if gpus is None else int(gpus)
        if n < 1:
            raise ValueError(f"--gpus must be >= 1 (got {n})")
        return ("spawn", n) if n > 1 else ("self", 1)
    world = int(ws)
    if gpus is not None and int(gpus) != world:
        raise ValueError(f"--gpus {gpus} disagrees with WORLD_SIZE={world} set by the launcher")
    return ("self", world)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_command(n, argv, port):
    """The torch.distributed.run command line that runs this file as n ranks
    on one node (rendezvous on 127.0.0.1; the container hostname may not
    resolve)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def spawn_ranks(n, argv):
    """Run n rank processes as children (this process has made no GPU call)
    and return their launcher's exit status."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL
    return subprocess.call(spawn_command(n, argv, _free_port()), env=env)


class ChamferStep:
    """Buffers + one hot-path step, all on the current stream.  The loss means
    of consecutive steps go to consecutive rows of `loss` ([slots, 2]), so the
    cross-rank all-reduce can take the losses of a whole graph of steps at once
    (one bucketed collective instead of one 8-byte collective per step)."""

    def __init__(self, dev, world, seed, slots, fused=True, variant=None):
        g = torch.Generator(device="cpu").manual_seed(seed)
        self.xyz1 = torch.rand(B, N, 3, generator=g).to(dev)
        self.xyz2 = torch.rand(B, M, 3, generator=g).to(dev)
        self.d1 = torch.empty(B, N, device=dev)
        self.d2 = torch.empty(B, M, device=dev)
        self.i1 = torch.empty(B, N, dtype=torch.int32, device=dev)
        self.i2 = torch.empty(B, M, dtype=torch.int32, device=dev)
        # gradient of mean() over the GLOBAL batch (world * B clouds)
        self.g1 = torch.full((B, N), 1.0 / (world * B * N), device=dev)
        self.g2 = torch.full((B, M), 1.0 / (world * B * M), device=dev)
        self.gx1 = torch.empty(B, N, 3, device=dev)
        self.gx2 = torch.empty(B, M, 3, device=dev)
        self.w1, self.w2 = 1.0 / (world * B * N), 1.0 / (world * B * M)
        self.loss = torch.zeros(slots, 3, device=dev)
        self.variant = variant
        if variant is not None:
            pcm_hip.load_tune_library()  # (workspace sized for the tuning build's variants too)
        self.ws = pcm_hip.chamfer_workspace(dev, B, N, M)
        self.world = world
        self.collective = dist.is_available() and dist.is_initialized()
        self.fused = fused and pcm_hip.loss_grad_supported(self.xyz1, self.xyz2)

    def __call__(self, slot=0):
        if self.fused:
            # one launch: forward, deterministic mean(dist1), mean(dist2), and both gradients
            pcm_hip.chamfer_loss_grad(self.xyz1, self.xyz2, self.w1, self.w2, self.d1, self.d2, self.i1,
                                      self.i2, self.loss[slot], self.gx1, self.gx2, self.ws, variant=self.variant)
            return
        # forward + deterministic in-kernel mean(dist1), mean(dist2); then the backward
        pcm_hip.chamfer_forward_loss(self.xyz1, self.xyz2, self.d1, self.d2, self.i1, self.i2,
                                     self.loss[slot], self.ws)
        pcm_hip.chamfer_backward(self.xyz1, self.xyz2, self.g1, self.g2, self.i1, self.i2,
                                 self.gx1, self.gx2)

    def launcher(self):
        """The step as direct launches through the C ABI (include/pcm.h), its
        arguments bound once: what a native training loop calls per step,
        without the Python wrapper's per-call checks (~10 us of host time
        against a ~14 us kernel).  The host stays ahead of the GPU, so the
        timed region holds back-to-back kernels and no replay floor."""
        import ctypes
        L = pcm_hip.load_library()
        P = pcm_hip._ptr
        st = pcm_hip._stream(self.xyz1.device)
        ci, cf, cs = ctypes.c_int, ctypes.c_float, ctypes.c_size_t
        if self.fused:
            # K steps = K calls of pcm_chamfer_loss_grad from one host call
            # (include/pcm.h pcm_chamfer_loss_grad_steps: a C loop over the
            # public entry; ctypes costs ~17 us per call of 17 arguments from
            # Python, more than the kernel, r05e)
            f = L.pcm_chamfer_loss_grad_steps
            f.restype = ctypes.c_int
            args = (P(self.xyz1), P(self.xyz2), ci(B), ci(N), ci(M), cf(self.w1), cf(self.w2), P(self.d1), P(self.d2),
                    P(self.i1), P(self.i2), P(self.loss[0]), P(self.gx1), P(self.gx2), P(self.ws),
                    cs(self.ws.numel()), st)

            def go(k=1):
                if f(ci(k), *args):
                    raise pcm_hip.PcmError("pcm_chamfer_loss_grad failed")
            return go
        f1, f2 = L.pcm_chamfer_forward_loss, L.pcm_chamfer_backward
        a1 = (P(self.xyz1), P(self.xyz2), ci(B), ci(N), ci(M), P(self.d1), P(self.d2), P(self.i1), P(self.i2),
              P(self.loss[0]), P(self.ws), cs(self.ws.numel()), st)
        a2 = (P(self.xyz1), P(self.xyz2), ci(B), ci(N), ci(M), P(self.g1), P(self.g2), P(self.i1), P(self.i2),
              P(self.gx1), P(self.gx2), st)

        def go2(k=1):
            for _ in range(k):
                if f1(*a1) or f2(*a2):
                    raise pcm_hip.PcmError("pcm_chamfer_forward_loss / pcm_chamfer_backward failed")
        return go2

    def reduce_losses(self, rows):
        """sum of per-rank means over RCCL (/world = global mean), stream-ordered"""
        if self.collective:
            dist.all_reduce(self.loss[:rows])


def time_region(fn, calls, dev, world, gpu=None):
    """Wall time of `calls` calls of fn, bracketed by a barrier + synchronize
    on both sides, max over ranks.  gpu (a list): HIP events recorded on the
    current stream at the region's edges append the GPU-side time (s)."""
    if dist.is_initialized():
        dist.barrier()
    s = torch.cuda.current_stream(dev)
    if gpu is not None:
        # the events exist and have been recorded once before the clock starts
        # (HIP creates an event at its first record: that first-use cost is
        # not the region's)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        e1.record(s)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if gpu is not None:
        e0.record(s)
    for _ in range(calls):
        fn()
    if gpu is not None:
        e1.record(s)
    torch.cuda.synchronize(dev)
    if dist.is_initialized():
        dist.barrier()
    t = time.perf_counter() - t0
    if gpu is not None:
        gpu.append(e0.elapsed_time(e1) * 1e-3)
    if dist.is_initialized():
        tt = torch.tensor([t], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt.item())
    return t


def kernel_avg_us(launch, reps, dev, graph=True):
    """Average device time of one launch: `reps` back-to-back launches captured
    in a hipGraph, replayed between two HIP events recorded on the stream the
    kernels run on (so the ~10 us host cost of a ctypes launch is not timed;
    the inter-kernel gap inside the graph is).  graph=False: eager launches."""
    s = torch.cuda.current_stream(dev)
    for _ in range(5):
        launch()
    run = lambda: [launch() for _ in range(reps)]  # noqa: E731
    if graph:
        cs = torch.cuda.Stream(dev)
        cs.wait_stream(s)
        with torch.cuda.stream(cs):
            launch()
        s.wait_stream(cs)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                launch()
        run = g.replay
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    run()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / reps


def reference_call_leg(dev, reps=50):
    """The call sequence the UNCHANGED caller runs, literally: train.py:163
    hands loss/loss.py a transposed view of the generator output,
    loss/loss.py:34-36 builds chamfer_3DDist, takes mean(dist1)+mean(dist2),
    and train.py:176 runs .backward() through chamfer_3DFunction
    (dist_chamfer_3D.py), at BASELINE config 2.  Timed eagerly (host launch
    cost included) and captured whole -- forward, means, autograd backward --
    into one hipGraph; the ratio is against the fused one-launch step."""
    sys.path.insert(0, os.path.join(PKG, "metric", "chamfer3D"))
    import dist_chamfer_3D
    g = torch.Generator(device="cpu").manual_seed(11)
    fake = torch.rand(B, 3, N, generator=g).to(dev).requires_grad_(True)  # generator output layout
    points = torch.rand(B, M, 3, generator=g).to(dev)

    def call():
        # gen.zero_grad() before total_loss.backward() (train.py:174-175): the
        # generator output's gradient is never accumulated into an older one
        # (fake stands in for it as a leaf here; without this every captured
        # call would add an accumulation kernel train.py does not run)
        fake.grad = None
        chamLoss = dist_chamfer_3D.chamfer_3DDist()
        dist1, dist2, idx1, idx2 = chamLoss(fake.transpose(2, 1), points)
        loss = torch.mean(dist1) + torch.mean(dist2)
        loss.backward()
        return loss

    def eager():
        call()

    s = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    side.wait_stream(s)
    with torch.cuda.stream(side):
        for _ in range(3):
            eager()
    s.wait_stream(side)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        eager()
    torch.cuda.synchronize(dev)
    eager_us = (time.perf_counter() - t0) * 1e6 / reps

    fake.grad = None
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(GRAPH_STEPS):
            call()  # grads accumulate into the graph's own .grad buffer; the time is what counts
    graph.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    k = max(1, reps // GRAPH_STEPS)
    e0.record(s)
    for _ in range(k):
        graph.replay()
    e1.record(s)
    e1.synchronize()
    graph_us = e0.elapsed_time(e1) * 1000.0 / (k * GRAPH_STEPS)
    pairs = 2 * B * N * M
    return {"sequence": "gen.zero_grad(); chamfer_3DDist()(fake.transpose(2,1), points); mean(dist1)+mean(dist2); "
                        ".backward() (loss/loss.py:34-36, train.py:163,174-175)",
            "eager_us_per_step": eager_us, "graph_us_per_step": graph_us,
            "graph_pairs_per_s": pairs / (graph_us * 1e-6)}


LAMBDA_CD = 100  # train.py:43 --lambda_cd default


def training_call_leg(dev, reps=50):
    """The call train.py makes through THIS build's loss (loss/loss.py
    counterpart): gen.zero_grad(), chamfer_loss =
    Loss().get_chamfer_loss(fake.transpose(2, 1), points), total_loss =
    chamfer_loss * lambda_cd (100), total_loss.backward() (train.py:163,169,
    174-176; the EMD term has its own legs), at BASELINE config 2 on the
    generator's [B, 3, N] output layout.  The one-launch step reads the
    transposed view in place and computes the lambda-weighted gradient (the
    scale learned from the previous step), the backward's rescale launch finds
    nothing to do.  Timed eagerly and as a captured 20-step graph."""
    sys.path.insert(0, os.path.join(PKG, "loss"))
    import loss as loss_mod
    g = torch.Generator(device="cpu").manual_seed(11)  # reference_call_leg's clouds
    fake = torch.rand(B, 3, N, generator=g).to(dev).requires_grad_(True)
    points = torch.rand(B, M, 3, generator=g).to(dev)
    loss_fn = loss_mod.Loss()

    def call():
        fake.grad = None  # gen.zero_grad()
        chamfer_loss = loss_fn.get_chamfer_loss(fake.transpose(2, 1), points)
        total_loss = chamfer_loss * LAMBDA_CD
        total_loss.backward()
        return total_loss

    out = _time_call(call, dev, reps)
    out["before"] = _time_call(lambda: _round5_training_call(fake, points), dev, reps)
    out["before"]["form"] = ("round 5's chamfer_3DLossFunction: .contiguous() copy of the transposed view, the "
                             "one-launch step at weight 1/(B N), the saved gradients multiplied by the upstream "
                             "gradient in backward (two torch multiplies)")
    out.update(sequence="gen.zero_grad(); Loss().get_chamfer_loss(fake.transpose(2,1), points) * lambda_cd(100); "
                        ".backward() (train.py:163,169,174-176, this build's loss/loss.py)",
               graph_pairs_per_s=2 * B * N * M / (out["graph_us_per_step"] * 1e-6),
               kernels_per_step="profiles/r06/training_call_kernels.txt (rocprofv3 kernel trace of "
                                "tools/training_call_trace.py)")
    return out


class _Round5LossFunction(torch.autograd.Function):
    """Round 5's form of the fused loss (for the training_call leg's 'before'
    figure only): rows copied, gradient at weight 1/(B N), scaled afterwards."""

    @staticmethod
    def forward(ctx, xyz1, xyz2):
        xyz1, xyz2 = xyz1.contiguous(), xyz2.contiguous()
        b, n, _ = xyz1.shape
        m = xyz2.shape[1]
        dev = xyz1.device
        d1, d2 = torch.empty(b, n, device=dev), torch.empty(b, m, device=dev)
        i1 = torch.empty(b, n, dtype=torch.int32, device=dev)
        i2 = torch.empty(b, m, dtype=torch.int32, device=dev)
        means = torch.empty(3, device=dev)
        g1, g2 = torch.empty_like(xyz1), torch.empty_like(xyz2)
        pcm_hip.chamfer_loss_grad(xyz1, xyz2, 1.0 / (b * n), 1.0 / (b * m), d1, d2, i1, i2, means, g1, g2)
        ctx.save_for_backward(g1, g2)
        return means[2]

    @staticmethod
    def backward(ctx, grad_loss):
        g1, g2 = ctx.saved_tensors
        return g1 * grad_loss, g2 * grad_loss


def _round5_training_call(fake, points):
    fake.grad = None
    total_loss = _Round5LossFunction.apply(fake.transpose(2, 1), points) * LAMBDA_CD
    total_loss.backward()
    return total_loss


def _time_call(call, dev, reps):
    """A python-level call sequence timed eagerly (host launch cost included)
    and as a captured GRAPH_STEPS-step graph (device time per step)."""
    s = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    side.wait_stream(s)
    with torch.cuda.stream(side):
        for _ in range(3):
            call()
    s.wait_stream(side)
    for _ in range(3):
        call()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        call()
    torch.cuda.synchronize(dev)
    eager_us = (time.perf_counter() - t0) * 1e6 / reps
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(GRAPH_STEPS):
            call()
    graph.replay()
    graph.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # warm replays for ~5 ms first: the eager loop above leaves the GPU mostly
    # idle, and the first few ms of load run its VALU-bound kernels slower
    # (DESIGN.md section 5); without them the leg's figure depended on which
    # legs ran before it (profiles/r06/tc_order_r06ze.txt)
    e0.record(s)
    graph.replay()
    e1.record(s)
    e1.synchronize()
    for _ in range(int(5.0 / max(e0.elapsed_time(e1), 1e-3)) + 1):
        graph.replay()
    k = max(5, reps // GRAPH_STEPS)
    e0.record(s)
    for _ in range(k):
        graph.replay()
    e1.record(s)
    e1.synchronize()
    graph_us = e0.elapsed_time(e1) * 1000.0 / (k * GRAPH_STEPS)
    return {"eager_us_per_step": eager_us, "graph_us_per_step": graph_us}


EMD_TRAIN_CLOUDS = os.path.join(REPO, "bench_data", "emd_training_call.npz")


def generator_predictions(dev):
    """The clouds a seeded random-init 3D-FENet generator predicts (train/fenet.py,
    the model train.py:160 runs; its RepVGG checkpoint is absent, so seeded
    weights) for synthetic images, and uniform [0,1) ground truth: the inputs
    the training call loss/loss.py:23 sees early in training.  Computed once on
    the CPU and committed (tools/make_emd_train_clouds.py), so the leg is the
    same workload on every box (a GPU forward's algorithm choice varies by box,
    and a 1-ulp change moves the auction)."""
    import numpy as np
    with np.load(EMD_TRAIN_CLOUDS) as z:
        pred, points = z["pred"], z["points"]
    return torch.from_numpy(pred).to(dev), torch.from_numpy(points).to(dev)


def emd_leg(dev, reps=10, eps=EMD_EPS, iters=EMD_ITERS, clouds=None, label="uniform [0,1) clouds, seeded"):
    """BASELINE config 3 by default; with eps=0.05, iters=3000 the training call
    of loss/loss.py:23.  The auction stops once every point is assigned, so
    both rates are given: iters_per_s counts the REQUESTED iterations (the
    reference launches all of them), active_iters_per_s the iterations that
    had bidders.  Roofline: the reference's work, every bidder scanning every
    object each iteration (emd_cuda.cu:139-155), in VALU lane-ops."""
    if clouds is None:
        g = torch.Generator(device="cpu").manual_seed(3)
        x1 = torch.rand(EMD_B, EMD_N, 3, generator=g).to(dev)
        x2 = torch.rand(EMD_B, EMD_N, 3, generator=g).to(dev)
    else:
        x1, x2 = clouds
    b, n, _ = x1.shape
    d = torch.empty(b, n, device=dev)
    a = torch.empty(b, n, dtype=torch.int32, device=dev)
    ws = pcm_hip.emd_workspace(dev, b, n)
    # counts (a separate, untimed run: the counters perturb the timing)
    st = torch.zeros(3 * iters + 16 + b, dtype=torch.int32, device=dev)
    pcm_hip.emd_forward(x1, x2, eps, iters, d, a, workspace=ws, stats=st, diag=1)
    torch.cuda.synchronize(dev)
    per = st[:2 * iters].view(iters, 2).cpu()
    active = int((per[:, 0] > 0).sum())
    bids = int(per[:, 0].sum())
    misses = int(per[:, 1].sum())  # cache misses; the reserve bids some of them without a full scan
    reserve_bids = int(st[2 * iters + 13].item())
    full_scans = misses - reserve_bids

    def run():
        pcm_hip.emd_forward(x1, x2, eps, iters, d, a, None, ws)

    us = kernel_avg_us(run, reps, dev, graph=False)  # >= 250 us launches: host cost hidden
    # elements whose master timed out on a helper job in the last timed forward
    # (the result stays exact, but the call fell back to master-only scans)
    timeouts = pcm_hip.emd_timeouts(ws, b, n)
    pairs = bids * n
    lane_ops = pairs * EMD_LANE_OPS_PER_PAIR / (us * 1e-6)
    return {"config": f"B={b} N=M={n} iters={iters} eps={eps}", "clouds": label,
            "ms_per_forward": us / 1000.0, "iters_requested": iters, "iters_run": active,
            "iters_per_s": iters / (us * 1e-6), "active_iters_per_s": active / (us * 1e-6),
            "bids": bids, "cache_misses": misses, "reserve_bids": reserve_bids, "full_scans": full_scans,
            "helper_timeouts": timeouts, "bid_pair_evals_per_s": pairs / (us * 1e-6),
            "roofline": {"bound": "valu", "kernel": "emd_seed_kernel + emd_auction_kernel",
                         "achieved": lane_ops / 1e12, "peak": VALU_LANE_OPS_PEAK / 1e12,
                         "unit": "T lane-ops/s", "frac": lane_ops / VALU_LANE_OPS_PEAK,
                         "note": f"{EMD_LANE_OPS_PER_PAIR} lane-ops per (bidder, object) pair the reference "
                                 "evaluates; the build evaluates fewer (caches), so this is the reference-work rate"},
            "roofline_executed": (emd_executed_roofline(us) if clouds is None and eps == EMD_EPS else
                                  emd_executed_roofline(us, "counters_emd_training_call")
                                  if clouds is not None and eps == 0.05 and iters == 3000 else None)}


# the EMD kernels as profile_kernels.py runs them (BASELINE config 3) in the committed PMC summary
EMD_KERNELS = ("emd_seed_kernel<true, true>", "emd_auction_kernel<false, true, true>")


def emd_executed_roofline(us, which="counters"):
    """The work the build actually executes: VALU wave instructions per
    forward (seed + auction, rocprofv3 SQ_INSTS_VALU from the committed PMC
    summary: "counters" = BASELINE config 3, "counters_emd_training_call" =
    the training call's own pass) x 64 lanes / this forward's time, against
    the 78.6 T lane-instruction issue ceiling; with the auction's wait share
    (SQ_WAIT_ANY / SQ_WAVE_CYCLES) and its busiest-wave view."""
    try:
        with open(PMC_SUMMARY) as fh:
            cnt = json.load(fh)[which]
        waves = sum(cnt[k]["SQ_INSTS_VALU"] for k in EMD_KERNELS)
        auc = cnt[EMD_KERNELS[1]]
        wait = auc["SQ_WAIT_ANY"] / auc["SQ_WAVE_CYCLES"] if "SQ_WAIT_ANY" in auc else None
    except (OSError, KeyError, ValueError, ZeroDivisionError):
        return None
    rate = waves * 64 / (us * 1e-6)
    return {"bound": "valu", "valu_wave_instructions": waves, "achieved": rate / 1e12,
            "peak": VALU_LANE_OPS_PEAK / 1e12, "unit": "T lane-ops/s", "frac": rate / VALU_LANE_OPS_PEAK,
            "auction_wait_share": wait, "source": os.path.relpath(PMC_SUMMARY, REPO) + ":" + which}


def chamfer_executed_roofline(kernel, us):
    """The one-launch kernel's executed VALU work: its counter VALU wave
    instructions per launch (rocprofv3 SQ_INSTS_VALU, committed PMC summary)
    x 64 lanes / this run's kernel time, against the 78.6 T lane-instruction
    issue ceiling -- what the VALU actually issued, beside the algorithmic
    8-FLOP-per-pair figure; with the counters' wait share."""
    try:
        with open(PMC_SUMMARY) as fh:
            c = json.load(fh)["counters"][kernel]
        waves = c["SQ_INSTS_VALU"]
        wait = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
    except (OSError, KeyError, ValueError, ZeroDivisionError):
        return None
    rate = waves * 64 / (us * 1e-6)
    return {"bound": "valu", "valu_wave_instructions": waves, "achieved": rate / 1e12,
            "peak": VALU_LANE_OPS_PEAK / 1e12, "unit": "T lane-ops/s", "frac": rate / VALU_LANE_OPS_PEAK,
            "wait_share": wait, "source": os.path.relpath(PMC_SUMMARY, REPO)}


def dense_f16_leg(dev, reps=10):
    """BASELINE config 5: dense Chamfer fwd+bwd, B=8, N=M=16384, fp16 clouds
    (fp32 arithmetic on the exactly-widened coordinates), graph-timed."""
    b, n = 8, 16384
    g = torch.Generator(device="cpu").manual_seed(5)
    x1 = torch.rand(b, n, 3, generator=g).half().to(dev)
    x2 = torch.rand(b, n, 3, generator=g).half().to(dev)
    d1, d2 = torch.empty(b, n, device=dev), torch.empty(b, n, device=dev)
    i1 = torch.empty(b, n, dtype=torch.int32, device=dev)
    i2 = torch.empty(b, n, dtype=torch.int32, device=dev)
    g1 = torch.full((b, n), 1.0 / (b * n), device=dev)
    g2 = torch.full((b, n), 1.0 / (b * n), device=dev)
    gx1 = torch.empty_like(x1)
    gx2 = torch.empty_like(x2)

    def fwd():  # the public path: clouds this large take the grid forward (csrc/chamfer_grid.hip)
        pcm_hip.chamfer_forward(x1, x2, d1, d2, i1, i2)

    L = pcm_hip.load_library()
    P = pcm_hip._ptr

    def fwd_dense():  # every pair evaluated (pcm_chamfer_forward_f16): the same outputs, bit for bit
        pcm_hip._check(L.pcm_chamfer_forward_f16(P(x1), P(x2), b, n, n, P(d1), P(d2), P(i1), P(i2),
                                                 pcm_hip._stream(dev)), "pcm_chamfer_forward_f16")

    def bwd():
        pcm_hip.chamfer_backward(x1, x2, g1, g2, i1, i2, gx1, gx2)

    f_us = kernel_avg_us(fwd, reps, dev)
    fd_us = kernel_avg_us(fwd_dense, reps, dev)
    b_us = kernel_avg_us(bwd, reps, dev)
    pairs = 2 * b * n * n
    # the grid search's executed screen work: every gathered candidate against
    # the 64 queries of its wave (csrc/chamfer_grid.hip per-wave stats)
    waves = b * 2 * ((n + 63) // 64)
    st = torch.zeros(waves * 12, dtype=torch.int32, device=dev)
    pcm_hip.tune_chamfer_forward_grid(x1, x2, d1, d2, i1, i2, stats=st)
    torch.cuda.synchronize(dev)
    evaluated = int(st[:waves * 4].view(waves, 4)[:, 2].long().sum().item()) * 64
    return {"config": f"B={b} N=M={n} fp16 clouds, fp32 arithmetic",
            # every pair evaluated: the dense filtered scan + the backward (round-3 meaning of the field)
            "pairs_per_s": pairs / ((fd_us + b_us) * 1e-6),
            "fwd_dense_scan_us": fd_us, "bwd_us": b_us,
            "dense_scan_fwd_tflops": pairs * FLOP_PER_PAIR / (fd_us * 1e-6) / 1e12,
            # the public path (clouds this large take the grid forward): same outputs bit for bit
            "grid": {"fwd_path": "grid (pcm_chamfer_forward_ws_f16)", "fwd_us": f_us,
                     "effective_pairs_per_s": pairs / ((f_us + b_us) * 1e-6),
                     "effective_note": "all-pairs equivalent, 2*B*N*M / (grid fwd + bwd): NOT a VALU rate",
                     "evaluated_pairs": evaluated, "evaluated_fraction": evaluated / pairs,
                     "evaluated_pairs_per_s": evaluated / (f_us * 1e-6)}}


ICP_B, ICP_N, ICP_PASSES = 32, 1024, 50


def icp_leg(dev, with_cpu, reps=3):
    """ICP alignment of B=32 prediction/ground-truth pairs of
    1024 points (testnet.py:62-64), whole loop in one launch; tolerance < 0 so
    every pair runs exactly ICP_PASSES passes (the reference default stops
    on convergence).  CPU side: the reference's algorithm (sklearn kd-tree NN,
    numpy SVD) restated in oracle/icp_oracle.py, on 2 pairs."""
    import numpy as np
    g = torch.Generator(device="cpu").manual_seed(7)
    A = (torch.randn(ICP_B, ICP_N, 3, generator=g, dtype=torch.float64) * 0.3).to(dev)
    B = A + 0.01 * torch.randn(ICP_B, ICP_N, 3, generator=g, dtype=torch.float64).to(dev)
    T = torch.empty(ICP_B, 4, 4, dtype=torch.float64, device=dev)
    d = torch.empty(ICP_B, ICP_N, dtype=torch.float64, device=dev)
    it = torch.empty(ICP_B, dtype=torch.int32, device=dev)

    def run():
        pcm_hip.icp(A, B, None, ICP_PASSES, -1.0, T, d, it)

    us = kernel_avg_us(run, reps, dev, graph=False)
    passes = ICP_B * ICP_PASSES
    pairs = passes * ICP_N * ICP_N
    out = {"config": f"B={ICP_B} pairs, N={ICP_N}, {ICP_PASSES} passes each (tolerance < 0), float64 decisions",
           "kernel": "icp_kernel", "ms_per_launch": us / 1000.0,
           "passes_per_s": passes / (us * 1e-6), "nn_pairs_per_s": pairs / (us * 1e-6),
           "screen_tflops": pairs * FLOP_PER_PAIR / (us * 1e-6) / 1e12}
    if with_cpu:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import icp_oracle  # CPU baseline leg only
        An, Bn = A[:2].cpu().numpy(), B[:2].cpu().numpy()
        t0 = time.perf_counter()
        for k in range(2):
            icp_oracle.icp(An[k], Bn[k], max_iterations=ICP_PASSES, tolerance=-1.0,
                           nn=icp_oracle.nearest_neighbor_sklearn)
        el = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": 2 * ICP_PASSES / el, "unit": "passes/s", "cores": 1, "kind": "port",
                               "sample": f"2 pairs x {ICP_PASSES} passes, utils/icp.py algorithm with sklearn "
                                         f"kd-tree NN (oracle/icp_oracle.py), {el:.2f} s"}
        out["speedup_vs_cpu"] = out["passes_per_s"] / out["cpu_baseline"]["value"]
    return out


def pmc_bytes(kernel):
    """HBM-side bytes per launch of `kernel` from the committed rocprofv3 PMC
    summary (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE), or None."""
    try:
        with open(PMC_SUMMARY) as fh:
            ent = json.load(fh)["counters"][kernel]
        return ent["hbm_bytes"]
    except (OSError, KeyError, ValueError):
        return None


def host_cores():
    """The CPU share this process may use: the scheduler affinity, capped by
    OMP_NUM_THREADS when set (the GPU box exports 16, its share of a larger
    host whose every core nproc would report)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline(target_s=8.0):
    """The oracle's C restatement of the reference O(N*M) loop (chamfer3D.cu:
    12-195 / utils/utils.py:246-266), OpenMP over (batch, query), on the FULL
    B=32 workload: the box's host cores (value) and one core (single_core)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np
    import oracle as O  # CPU baseline leg only
    O.build()
    rng = np.random.default_rng(0)
    a = rng.random((B, N, 3), dtype=np.float32)
    c = rng.random((B, M, 3), dtype=np.float32)
    g1 = np.full((B, N), 1.0 / (B * N), np.float32)
    g2 = np.full((B, M), 1.0 / (B * M), np.float32)

    def timed(threads, budget):
        reps, t0 = 0, time.perf_counter()
        while True:
            d1, d2, i1, i2 = O.chamfer_forward(a, c, nthreads=threads)
            O.chamfer_backward(a, c, g1, g2, i1, i2, nthreads=threads)
            reps += 1
            el = time.perf_counter() - t0
            if el >= budget or reps >= 10000:
                return reps, el

    threads = host_cores()
    reps, el = timed(threads, target_s)
    reps1, el1 = timed(1, target_s / 2)
    pairs = 2 * B * N * M
    return {"value": pairs * reps / el, "unit": "point-pairs/s", "cores": threads, "kind": "port",
            "sample": f"{reps} reps of the full Chamfer fwd+bwd workload (B={B}, N=M={N}), oracle/pcm_oracle.c, "
                      f"OpenMP {threads} threads (the box's CPU share), {el:.1f} s",
            "single_core": {"value": pairs * reps1 / el1, "unit": "point-pairs/s", "cores": 1,
                            "sample": f"{reps1} reps of the same workload on 1 thread, {el1:.1f} s"}}


def capture_steps(step, per, dev, world, allreduce):
    """One hipGraph of `per` consecutive steps.  With `allreduce`, every step's
    own loss row is all-reduced right after its kernel, on a side stream that
    forks from the step and joins at the end of the graph, so the collective
    of step i overlaps the kernel of step i+1 (the loss is reported, nothing
    in the next step reads it)."""
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream(dev) if allreduce else None
    if allreduce:
        # no collective in flight for the process group's watchdog to query
        # while the capture runs; thread_local: its event queries are legal
        torch.cuda.synchronize(dev)
        dist.barrier()
    with torch.cuda.graph(g, capture_error_mode="thread_local" if allreduce else "global"):
        cur = torch.cuda.current_stream(dev)
        for i in range(per):
            step(i)
            if allreduce:
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    dist.all_reduce(step.loss[i])
        if allreduce:
            cur.wait_stream(side)
    return g


def warm_graphs(g_many, g_one, per, warmup, steps, run_steps, dev, world):
    """Warmup of the timed region's own graphs: whole replays of the very
    `per`-step graph the timed region replays (so its first replay -- graph
    upload, first touch of its kernels' arguments -- is paid here, never
    timed), plus the one-step graph when `steps` is not a multiple of `per`.
    At least `warmup` steps run (rounded up to whole replays; the count is
    reported).  Returns the graph facts for the JSON line."""
    info = {"graph_steps": per, "warmup_steps_requested": warmup}
    ran = 0
    if g_many is not None and warmup > 0:
        reps = -(-warmup // per)
        info["first_replay_us"] = time_region(g_many.replay, 1, dev, world) * 1e6
        for _ in range(reps - 1):
            g_many.replay()
        ran = reps * per
        if steps % per and g_one is not None:
            g_one.replay()
            ran += 1
    elif warmup > 0:
        run_steps(warmup)
        ran = warmup
    torch.cuda.synchronize(dev)
    info["warmup_steps_run"] = ran
    return info


def sustained_kernel_us(launch, dev, busy_ms=45.0, reps=200):
    """Per-launch device time once the GPU has run the step back to back for
    `busy_ms` (profiles/r06/clock_state_r06k.txt: after an idle second the
    step takes 15.1-15.3 us per launch and settles at 13.5 us after ~30 ms of
    load; the in-kernel stamps put the whole difference in the VALU-bound scan,
    profiles/r06/stamps_warm_cold_r06k.txt).  Reported beside the headline,
    never as it: the driver's 25-step command always runs in the first state."""
    s = torch.cuda.current_stream(dev)
    g = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream(dev)
    cs.wait_stream(s)
    with torch.cuda.stream(cs):
        launch()
    s.wait_stream(cs)
    with torch.cuda.graph(g):
        for _ in range(reps):
            launch()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    g.replay()
    e1.record(s)
    e1.synchronize()
    per_replay_ms = max(e0.elapsed_time(e1), 1e-3)
    for _ in range(int(busy_ms / per_replay_ms) + 1):  # queued back to back, no host gap
        g.replay()
    e0.record(s)
    for _ in range(5):
        g.replay()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / (5 * reps)


def side_legs(args, dev, rank, world):
    """The legs reported beside the headline (ICP, the unchanged caller's call
    sequence, config 5, EMD), after the headline (default) or, with
    --side-legs first, before its warmup.  Tried because back-to-back regions
    speed up ~9% over the first ~4 ms of load (profiles/r05/probe_events_r05j.txt);
    legs-first was not faster on the same box (r05o), so it is not the default."""
    side = {}
    if not args.no_icp:  # first: its CPU-timed part leaves the GPU idle
        side["icp"] = icp_leg(dev, with_cpu=rank == 0 and world == 1 and not args.no_cpu)
    if not args.no_ref_call:
        side["reference_call"] = reference_call_leg(dev)
        side["training_call"] = training_call_leg(dev)
    if not args.no_dense:
        side["dense_fp16"] = dense_f16_leg(dev)
    if not args.no_emd:
        side["emd"] = emd_leg(dev)
        pred, points = generator_predictions(dev)
        side["emd_training_call"] = emd_leg(dev, reps=3, eps=0.05, iters=3000, clouds=(pred, points),
                                            label="seeded random-init generator predictions vs uniform GT "
                                                  "(committed, bench_data/emd_training_call.npz)")
        side["emd_training_call_uniform"] = emd_leg(dev, reps=3, eps=0.05, iters=3000)
    torch.cuda.synchronize(dev)
    return side


def main(argv=None):
    args = parse(argv)
    # decided before any GPU call: a process that has initialised the GPU
    # must not start the ranks
    how, world = resolve_launch(args.gpus, os.environ)
    if how == "spawn":
        sys.exit(spawn_ranks(world, sys.argv[1:] if argv is None else argv))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one GPU per rank; a rehearsal with more ranks than GPUs (gloo) shares them
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    multi = world > 1 or args.force_dist
    if multi:
        if "MASTER_ADDR" not in os.environ:  # --force-dist without a launcher: a one-rank group
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0",
                              WORLD_SIZE="1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    per = 1 if args.eager else max(1, min(GRAPH_STEPS, args.steps))
    step = ChamferStep(dev, world, seed=BENCH_SEED + rank, slots=per, fused=not args.two_launch,
                       variant=args.tune_variant)

    def run_eager(k):
        for _ in range(k):
            step(0)
            step.reduce_losses(1)

    # a few eager steps before any capture (workspace allocation, first-call
    # costs); with --eager these are the warmup
    run_eager(args.warmup if args.eager else min(args.warmup, 3))
    torch.cuda.synchronize(dev)
    run_steps, mode, capture_error = run_eager, "eager, one all-reduce per step" if multi else "eager", None
    g_one = None
    graph_info = None
    if not args.eager:
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for i in range(3):
                step(i % per)
        torch.cuda.current_stream(dev).wait_stream(s)
        g_one = capture_steps(step, 1, dev, world, False)
        g_many = None
        if not multi:
            # `per` consecutive steps per hipGraph replay: the same form as at
            # N > 1 minus the per-step collective (round 6: the matched A/B of
            # this against K direct launches from a C loop gave 15.71 against
            # 15.82 us per step at K = 20, profiles/r06/ab_launch_form_r06c.txt)
            g_many = capture_steps(step, per, dev, world, False)
            if not args.c_loop:
                def run_steps(k):
                    for _ in range(k // per):
                        g_many.replay()
                    for _ in range(k % per):
                        g_one.replay()
                mode = f"hipgraph ({per} steps per graph; N>1 adds each step's all-reduce to the same graph)"
            else:
                go = step.launcher()

                def run_steps(k):
                    go(k)
                mode = ("direct launches, one per step: a C loop over pcm_chamfer_loss_grad with its arguments "
                        "bound once (pcm_chamfer_loss_grad_steps)")
        else:
            g_ar_many = g_ar_one = None
            if args.dist_backend == "nccl" and not args.eager_allreduce:
                try:
                    g_ar_many = capture_steps(step, per, dev, world, True)
                    g_ar_one = capture_steps(step, 1, dev, world, True)
                    # the captured collective must produce the all-reduced losses
                    g_ar_many.replay()
                    got = step.loss.clone()
                    for i in range(per):
                        step(i)
                    dist.all_reduce(step.loss)
                    if not torch.allclose(got, step.loss, rtol=1e-6, atol=0.0):
                        raise RuntimeError(f"captured all-reduce gave {got[0].tolist()}, eager "
                                           f"{step.loss[0].tolist()}")
                except Exception as e:  # noqa: BLE001 -- fall back to the eager per-step collective
                    capture_error = f"{type(e).__name__}: {e}"
                    g_ar_many = g_ar_one = None
                    torch.cuda.synchronize(dev)
                # every rank takes the same form: captured only if it worked everywhere
                ok = torch.tensor([0 if g_ar_many is None else 1], device=dev, dtype=torch.int32)
                dist.all_reduce(ok, op=dist.ReduceOp.MIN)
                if int(ok.item()) == 0:
                    if capture_error is None:
                        capture_error = "the captured collective failed on another rank"
                    g_ar_many = g_ar_one = None
            if g_ar_many is not None:
                g_many = g_ar_many

                def run_steps(k):
                    for _ in range(k // per):
                        g_ar_many.replay()
                    for _ in range(k % per):
                        g_ar_one.replay()
                mode = (f"hipgraph ({per} steps per graph, each step's loss all-reduced over RCCL inside "
                        "the graph on a side stream)")
            else:
                def run_steps(k):
                    for _ in range(k):
                        g_one.replay()
                        step.reduce_losses(1)
                mode = "one-step hipgraph replay + eager all-reduce of the step's loss, every step"
        side = side_legs(args, dev, rank, world) if args.side_legs == "first" else {}
        if multi or not args.c_loop:
            g_tail = g_one if not multi else (g_ar_one if g_ar_many is not None else None)
            graph_info = warm_graphs(g_many, g_tail, per, args.warmup, args.steps, run_steps, dev, world)
        else:
            g_many.replay()  # the graph form's first replay, outside every timed region
            torch.cuda.synchronize(dev)
            # then the timed region's own launches: W of them, last before the region
            run_steps(args.warmup)
            torch.cuda.synchronize(dev)
            graph_info = {"graph_steps": per, "warmup_steps_requested": args.warmup,
                          "warmup_steps_run": args.warmup}

    if args.eager:
        side = side_legs(args, dev, rank, world) if args.side_legs == "first" else {}
        run_steps(args.warmup)
        torch.cuda.synchronize(dev)
    gpu_t = []
    t = time_region(lambda: run_steps(args.steps), 1, dev, world, gpu=gpu_t)
    if graph_info is not None and g_many is not None:
        # a steady replay of the `per`-step graph after the timed region (with
        # --graph, compare with the first replay, which warmup paid)
        graph_info["steady_replay_us"] = time_region(g_many.replay, 1, dev, world) * 1e6
        graph_info["steady_replay_us_per_step"] = graph_info["steady_replay_us"] / per
    pairs_per_step = 2 * B * N * M
    value = world * args.steps * pairs_per_step / t
    ms = t * 1000.0 / args.steps

    # dominant kernel: the step's Chamfer forward (fused-loss) launch, timed on its stream
    fwd_us = kernel_avg_us(lambda: pcm_hip.chamfer_forward_loss(
        step.xyz1, step.xyz2, step.d1, step.d2, step.i1, step.i2, step.loss[0], step.ws), 200, dev)
    bwd_us = kernel_avg_us(lambda: pcm_hip.chamfer_backward(step.xyz1, step.xyz2, step.g1, step.g2,
                                                            step.i1, step.i2, step.gx1, step.gx2),
                           200, dev)
    fwd_tflops = pairs_per_step * FLOP_PER_PAIR / (fwd_us * 1e-6) / 1e12
    # the dominant kernel's duration: HIP events on the kernel's stream over
    # the timed region itself (back-to-back launches: the kernel plus its
    # launch boundary); the 200-launch graph average beside it
    region_us = gpu_t[0] * 1e6 / args.steps
    if step.fused:
        dom_kernel, dom_bytes = FUSED_KERNEL, FUSED_BYTES
        graph_kernel_us = kernel_avg_us(lambda: step(0), 200, dev)
        sustained_us = sustained_kernel_us(lambda: step(0), dev)
        dom_us = region_us if not (args.eager or multi) else graph_kernel_us
    else:
        dom_kernel, dom_bytes, dom_us = FWD_KERNEL, FWD_BYTES, fwd_us
        graph_kernel_us = fwd_us
        sustained_us = None
    dom_tflops = pairs_per_step * FLOP_PER_PAIR / (dom_us * 1e-6) / 1e12
    traffic = pmc_bytes(dom_kernel)
    out = {
        "metric": "Chamfer3D fwd+bwd point-pairs/sec @ B=32 N=M=1024; EMD iters/sec",
        "value": value,
        "unit": "point-pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: torch.rand uniform [0,1) clouds, seeded",
        "config": {"workload": "Chamfer3D fwd+bwd (+loss sums, +RCCL all-reduce of every step's loss when N>1)",
                   "batch_per_gpu": B, "n_points": N, "m_points": M,
                   "global_batch": world * B, "parallelism": f"dp{world} (batch-sharded)",
                   "launch": mode, "dist_backend": args.dist_backend if multi else None,
                   **({"tune_variant": args.tune_variant} if args.tune_variant is not None else {})},
        "roofline": {"bound": "valu", "kernel": dom_kernel,
                     "achieved": dom_tflops, "peak": FP32_VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": dom_tflops / FP32_VALU_PEAK_TFLOPS, "traffic": traffic,
                     "traffic_unit": "bytes/launch (rocprofv3 FETCH_SIZE*2+WRITE_SIZE, " +
                                     os.path.relpath(PMC_SUMMARY, REPO) + ")",
                     "kernel_us": dom_us, "kernel_us_source": (
                         "HIP events on the kernel's stream around the timed region, per step"
                         if dom_us == region_us else "HIP events around a 200-launch hipGraph replay, per launch"),
                     "kernel_us_graph200": graph_kernel_us, "timed_region_gpu_us_per_step": region_us,
                     "kernel_us_sustained": sustained_us,
                     "frac_sustained": None if sustained_us is None else
                     pairs_per_step * FLOP_PER_PAIR / (sustained_us * 1e-6) / 1e12 / FP32_VALU_PEAK_TFLOPS,
                     "sustained_note": "kernel_us_sustained: per launch after ~45 ms of back-to-back steps (a GPU "
                                       "busy as in a training loop); the headline's short region runs on a GPU "
                                       "that was idle, whose VALU-bound scan is ~25% slower (DESIGN.md section 5)",
                     "note": "FLOPs = 8 per point pair (algorithmic); VALU-bound, see DESIGN.md"},
        "roofline_hbm": {"bound": "hbm", "kernel": dom_kernel, "rank": rank,
                         "achieved": dom_bytes / (dom_us * 1e-6) / 1e9, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s",
                         "frac": dom_bytes / (dom_us * 1e-6) / 1e9 / HBM_PEAK_GBS,
                         "algorithmic_bytes": dom_bytes, "traffic": traffic,
                         "counter_achieved": None if traffic is None else traffic / (dom_us * 1e-6) / 1e9,
                         "counter_frac": None if traffic is None else traffic / (dom_us * 1e-6) / 1e9 / HBM_PEAK_GBS,
                         "note": "achieved = algorithmic bytes / kernel time; counter_achieved = rocprofv3 HBM-side "
                                 "bytes per launch / this rank's kernel time"},
        "two_launch": {"fwd_loss_kernel": FWD_KERNEL, "fwd_loss_us": fwd_us,
                       "fwd_tflops": fwd_tflops, "fwd_traffic": pmc_bytes(FWD_KERNEL),
                       "bwd_kernel": BWD_KERNEL, "bwd_us": bwd_us,
                       "bwd_achieved_gbs": BWD_BYTES / (bwd_us * 1e-6) / 1e9,
                       "bwd_algorithmic_bytes": BWD_BYTES, "bwd_traffic": pmc_bytes(BWD_KERNEL),
                       "step_us": fwd_us + bwd_us},
    }
    if graph_info is not None:
        out["graph"] = graph_info
        out["warmup_steps_run"] = graph_info["warmup_steps_run"]
    out["roofline"]["step_minus_kernel_us"] = ms * 1000.0 - dom_us
    out["roofline_executed"] = chamfer_executed_roofline(dom_kernel, dom_us)
    if capture_error is not None:
        out["config"]["allreduce_capture_error"] = capture_error
    if multi:
        # the other forms of the loss collective, beside the headline
        per_rank_us = torch.tensor([dom_us], device=dev, dtype=torch.float64)
        dist.all_reduce(per_rank_us, op=dist.ReduceOp.MAX)
        out["roofline"]["kernel_us_max_over_ranks"] = float(per_rank_us.item())

        def eager_per_step(k):
            for _ in range(k):
                (g_one.replay() if g_one is not None else step(0))
                dist.all_reduce(step.loss[0])
        eager_per_step(3)
        t_ps = time_region(lambda: eager_per_step(args.steps), 1, dev, world)
        out["eager_per_step_allreduce"] = {
            "launch": f"one-step hipgraph replay + eager {'RCCL' if args.dist_backend == 'nccl' else args.dist_backend} "
                      "all-reduce of the step's loss, every step",
            "ms_per_step": t_ps * 1000.0 / args.steps,
            "value": world * args.steps * pairs_per_step / t_ps}
        if not args.eager:
            g_bucket = capture_steps(step, per, dev, world, False)

            def bucketed(k):
                for _ in range(k // per):
                    g_bucket.replay()
                    step.reduce_losses(per)
            bucketed(per)
            kb = max(per, args.steps // per * per)
            t_b = time_region(lambda: bucketed(kb), 1, dev, world)
            out["bucketed_allreduce"] = {
                "launch": f"hipgraph of {per} steps, then ONE all-reduce of their {per} loss rows",
                "ms_per_step": t_b * 1000.0 / kb,
                "value": world * kb * pairs_per_step / t_b}
    if args.side_legs == "last":
        side = side_legs(args, dev, rank, world)
    out.update(side)
    if "reference_call" in out:
        out["reference_call"]["graph_vs_fused_step"] = out["reference_call"]["graph_us_per_step"] / (ms * 1000.0)
    if "training_call" in out:
        out["training_call"]["graph_vs_fused_step"] = out["training_call"]["graph_us_per_step"] / (ms * 1000.0)
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if multi:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
