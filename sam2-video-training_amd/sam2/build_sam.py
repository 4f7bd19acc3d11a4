"""sam2.build_sam (upstream) -> sam2_video.predictor.build_sam2_video_predictor"""
from sam2_video.predictor import build_sam2_video_predictor  # noqa: F401
