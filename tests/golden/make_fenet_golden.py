"""Generate tests/golden/fenet_golden.npz from the REFERENCE generator (run here, not on the GPU box).

Imports the reference's models/repvgg_edge_nose_NEW_cmlp.py read-only (with
PYTHONDONTWRITEBYTECODE so nothing is written into /root/reference), builds
its ``generator`` in training mode with the RepVGG-A2 body but WITHOUT the
absent checkpoint (``create_RepVGG_A2`` at :349-353 loads
../pretrained_models/RepVGG-A2-train.pth, which does not exist here: the
RepVGG constructor it wraps is called directly instead), loads the weights of
this build's ``fenet.Generator`` after ``seeded_init`` (renamed to the
reference's parameter names), and records the reference forward on a seeded
image batch.  The reference's forward calls ``.cuda()`` (:13, :21, :271);
this CPU-only container has no device, so ``Tensor.cuda``/``Module.cuda``
are made identity functions for the duration of this script.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_fenet_golden.py
"""
import os
import re
import sys

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_MODELS = "/root/reference/models"
SEED, B = 7, 2


def ref_name(mine: str) -> str:
    """This build's parameter/buffer name -> the reference generator's."""
    n = mine
    n = n.replace("encoder.stage0.", "RepVGG.stage0.")
    n = re.sub(r"^encoder\.stages\.(\d+)\.", lambda m: f"RepVGG.stage{int(m.group(1)) + 1}.", n)
    n = n.replace("encoder.linear.", "RepVGG.linear.")
    n = n.replace("edge_linear.", "linear.")
    n = n.replace(".dense.0.", ".rbr_dense.conv.").replace(".dense.1.", ".rbr_dense.bn.")
    n = n.replace(".point.0.", ".rbr_1x1.conv.").replace(".point.1.", ".rbr_1x1.bn.")
    n = n.replace(".skip.", ".rbr_identity.")
    return n


def main():
    sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "train"))
    import fenet
    torch.Tensor.cuda = lambda self, *a, **k: self
    torch.nn.Module.cuda = lambda self, *a, **k: self
    sys.path.insert(0, REF_MODELS)
    import repvgg_edge_nose_NEW_cmlp as ref

    ref.create_RepVGG_A2 = lambda deploy=False: ref.RepVGG(
        num_blocks=[2, 4, 14, 1], num_classes=1000, width_multiplier=[1.5, 1.5, 1.5, 2.75],
        override_groups_map=None, deploy=deploy)
    rgen = ref.generator(num_points=1024)
    mine = fenet.seeded_init(fenet.Generator(1024), SEED)
    sd = {ref_name(k): v for k, v in mine.state_dict().items()}
    missing, unexpected = rgen.load_state_dict(sd, strict=True), None
    del missing, unexpected
    n_ref = sum(p.numel() for p in rgen.parameters())
    rgen.train()
    g = torch.Generator().manual_seed(SEED)
    img = torch.rand(B, 3, 128, 128, generator=g) * 2 - 1  # Normalize([.5]*3, [.5]*3) range
    with torch.no_grad():
        p1, p2, p3 = rgen(img)
    np.savez_compressed(os.path.join(HERE, "fenet_golden.npz"), seed=SEED, img=img.numpy(),
                        pc1=p1.numpy(), pc2=p2.numpy(), pc3=p3.numpy(), n_params=n_ref)
    print("reference generator params", n_ref, "outputs", p1.shape, p2.shape, p3.shape)


if __name__ == "__main__":
    main()
