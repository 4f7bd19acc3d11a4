"""Upstream-`sam2` import paths the reference's evaluation uses (sam2_video/eval/inference.py:16
`from sam2.build_sam import build_sam2_video_predictor`), served by this build's
sam2_video.predictor on the libsam2hip kernels.  Only the video-predictor entry points exist."""
