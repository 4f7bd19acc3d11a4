"""Diagnostic (not a test): block-by-block comparison of the HIP image encoder against the
CPU oracle on the same weights/inputs.  python tests/debug_modules.py [size] [image_size]"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import sam2_oracle as O  # noqa: E402
from step_harness import build_model  # noqa: E402
from sam2_video.data.synthetic import make_clip  # noqa: E402
from sam2_video.kernels import ops  # noqa: E402
from sam2_video.model.configs import model_config  # noqa: E402
from sam2_video.utils.init import synth_tensor  # noqa: E402

size = sys.argv[1] if len(sys.argv) > 1 else "tiny"
S = int(sys.argv[2]) if len(sys.argv) > 2 else 256
cfg = model_config(size, S)
P = O.make_params(O.param_shapes(cfg), [], synth_tensor, seed=0)
orc = O.OracleSAM2(cfg, P)
model = build_model(size, S, [], dtype="fp32")
clip = make_clip(7, 2, S, 4, 2)
img = clip["images"]


def cmp(tag, got_nhwc, ref_nchw_or_nhwc, nhwc=True):
    g = got_nhwc.detach().float().cpu()
    r = ref_nchw_or_nhwc if nhwc else ref_nchw_or_nhwc.permute(0, 2, 3, 1)
    print(f"{tag:40s} maxdiff {(g - r).abs().max().item():.3e} scale {r.abs().max().item():.3e}")


trunk = model.image_encoder.trunk
x = img.permute(0, 2, 3, 1).contiguous().cuda()
xe = trunk.patch_embed(x)
ref = F.conv2d(img, P["image_encoder.trunk.patch_embed.proj.weight"], P["image_encoder.trunk.patch_embed.proj.bias"],
               stride=4, padding=3).permute(0, 2, 3, 1)
cmp("patch_embed", xe, ref)
from sam2_video.kernels.functional_sam import hiera_pos_embed  # noqa: E402
pe = hiera_pos_embed(trunk.pos_embed, trunk.pos_embed_window, xe.shape[1], xe.shape[2], torch.float32)
h, w = xe.shape[1:3]
rpe = F.interpolate(P["image_encoder.trunk.pos_embed"], size=(h, w), mode="bicubic")
win = P["image_encoder.trunk.pos_embed_window"]
rpe = (rpe + win.tile([a // b for a, b in zip(rpe.shape, win.shape)])).permute(0, 2, 3, 1)[0]
cmp("pos_embed", pe, rpe)
xr = ref + rpe
xg = ops.add_bcast(xe, pe)
for i, (blk, b) in enumerate(zip(trunk.blocks, orc.blocks)):
    xr = orc.hiera_block(xr, i, b)
    xg_in = xg
    xg = blk(xg_in)
    cmp(f"block {i} ws={b['ws']} qpool={b['q_pool']} dim={b['dim']}->{b['dim_out']} h={b['heads']}", xg, xr)
    xg = xr.cuda().contiguous()  # re-sync to isolate per-block error
