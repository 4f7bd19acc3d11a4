"""MI355X-native SAM2 video fine-tuning step (drop-in for yangkunyi/sam2-video-training's
`sam2_video` package on the training hot path).

Host code is Python on PyTorch-ROCm (allocation, streams, autograd plumbing,
torch.distributed); every arithmetic op of the step runs in `libsam2hip.so`
(hand-written gfx950 kernels behind a C ABI, see `include/sam2hip.h`).
"""
__version__ = "0.1.0"
