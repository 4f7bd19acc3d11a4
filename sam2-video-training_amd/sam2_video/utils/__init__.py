"""Utilities aggregator (reference sam2_video/utils/__init__.py).  The W&B GIF
visualisation of the reference is out of scope (logging side effect)."""
from .masks import cat_to_obj_mask, find_connected_components, merge_object_results_to_category
from .model_utils import (count_total_parameters, count_trainable_parameters, freeze_module_by_name,
                          get_model_info, get_trainable_module_names, save_model_config, setup_trainable_modules,
                          unfreeze_module_by_name)
from .prompts import generate_box_prompt, generate_point_prompt

__all__ = ["generate_point_prompt", "generate_box_prompt", "find_connected_components", "cat_to_obj_mask",
           "merge_object_results_to_category", "count_trainable_parameters", "count_total_parameters",
           "get_model_info", "setup_trainable_modules", "freeze_module_by_name", "unfreeze_module_by_name",
           "get_trainable_module_names", "save_model_config"]
