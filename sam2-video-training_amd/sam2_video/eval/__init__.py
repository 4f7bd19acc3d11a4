"""Evaluation metrics (reference sam2_video/eval): IoU / Dice / MAE on category-merged masks."""
