"""sam2.sam2_video_predictor (upstream) -> sam2_video.predictor.SAM2VideoPredictor"""
from sam2_video.predictor import SAM2VideoPredictor  # noqa: F401
