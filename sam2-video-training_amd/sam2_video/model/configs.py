"""Model configurations as Hydra-style dicts (`_target_` + kwargs).

They follow the schema of the reference's model YAML
(configs/sam2/sam2.1_hiera_t.yaml:5-121) so one resolver handles both: a user's
own YAML passed as `config_path`, or these named sizes (Hiera-T / B+ / L with
the SAM2.1 trunk hyper-parameters quoted in SURVEY.md §8(c)).  Pure Python (the
golden-fixture generator loads this file by path).
"""
from __future__ import annotations

import copy

_BASE = {
    "_target_": "sam2.modeling.sam2_base.SAM2Base",
    "image_encoder": {
        "_target_": "sam2.modeling.backbones.image_encoder.ImageEncoder",
        "scalp": 1,
        "trunk": {"_target_": "sam2.modeling.backbones.hieradet.Hiera"},
        "neck": {
            "_target_": "sam2.modeling.backbones.image_encoder.FpnNeck",
            "position_encoding": {
                "_target_": "sam2.modeling.position_encoding.PositionEmbeddingSine",
                "num_pos_feats": 256, "normalize": True, "scale": None, "temperature": 10000,
            },
            "d_model": 256,
            "fpn_top_down_levels": [2, 3],
            "fpn_interp_model": "nearest",
        },
    },
    "memory_attention": {
        "_target_": "sam2.modeling.memory_attention.MemoryAttention",
        "d_model": 256,
        "pos_enc_at_input": True,
        "layer": {
            "_target_": "sam2.modeling.memory_attention.MemoryAttentionLayer",
            "activation": "relu", "dim_feedforward": 2048, "dropout": 0.1, "pos_enc_at_attn": False,
            "self_attention": {
                "_target_": "sam2.modeling.sam.transformer.RoPEAttention",
                "rope_theta": 10000.0, "feat_sizes": [64, 64], "embedding_dim": 256, "num_heads": 1,
                "downsample_rate": 1, "dropout": 0.1,
            },
            "d_model": 256, "pos_enc_at_cross_attn_keys": True, "pos_enc_at_cross_attn_queries": False,
            "cross_attention": {
                "_target_": "sam2.modeling.sam.transformer.RoPEAttention",
                "rope_theta": 10000.0, "feat_sizes": [64, 64], "rope_k_repeat": True, "embedding_dim": 256,
                "num_heads": 1, "downsample_rate": 1, "dropout": 0.1, "kv_in_dim": 64,
            },
        },
        "num_layers": 4,
    },
    "memory_encoder": {
        "_target_": "sam2.modeling.memory_encoder.MemoryEncoder",
        "out_dim": 64,
        "position_encoding": {
            "_target_": "sam2.modeling.position_encoding.PositionEmbeddingSine",
            "num_pos_feats": 64, "normalize": True, "scale": None, "temperature": 10000,
        },
        "mask_downsampler": {
            "_target_": "sam2.modeling.memory_encoder.MaskDownSampler", "kernel_size": 3, "stride": 2, "padding": 1,
        },
        "fuser": {
            "_target_": "sam2.modeling.memory_encoder.Fuser",
            "layer": {
                "_target_": "sam2.modeling.memory_encoder.CXBlock",
                "dim": 256, "kernel_size": 7, "padding": 3, "layer_scale_init_value": 1e-6, "use_dwconv": True,
            },
            "num_layers": 2,
        },
    },
    "num_maskmem": 7,
    "image_size": 512,
    "sigmoid_scale_for_mem_enc": 20.0,
    "sigmoid_bias_for_mem_enc": -10.0,
    "use_mask_input_as_output_without_sam": True,
    "directly_add_no_mem_embed": True,
    "no_obj_embed_spatial": True,
    "use_high_res_features_in_sam": True,
    "multimask_output_in_sam": False,
    "iou_prediction_use_sigmoid": True,
    "use_obj_ptrs_in_encoder": True,
    "add_tpos_enc_to_obj_ptrs": True,
    "proj_tpos_enc_in_obj_ptrs": True,
    "use_signed_tpos_enc_to_obj_ptrs": True,
    "only_obj_ptrs_in_the_past_for_eval": True,
    "pred_obj_scores": True,
    "pred_obj_scores_mlp": True,
    "fixed_no_obj_ptr": True,
    "multimask_output_for_tracking": False,
    "use_multimask_token_for_obj_ptr": False,
    "multimask_min_pt_num": 0,
    "multimask_max_pt_num": 1,
    "use_mlp_for_obj_ptr_proj": True,
    "compile_image_encoder": False,
}

# Hiera trunk hyper-parameters per size (SAM2.1 releases).
TRUNKS = {
    "tiny": dict(embed_dim=96, num_heads=1, stages=[1, 2, 7, 2], global_att_blocks=[5, 7, 9],
                 window_pos_embed_bkg_spatial_size=[7, 7]),
    "small": dict(embed_dim=96, num_heads=1, stages=[1, 2, 11, 2], global_att_blocks=[7, 10, 13],
                  window_pos_embed_bkg_spatial_size=[7, 7]),
    "base_plus": dict(embed_dim=112, num_heads=2),
    "large": dict(embed_dim=144, num_heads=2, stages=[2, 6, 36, 4], global_att_blocks=[23, 33, 43],
                  window_pos_embed_bkg_spatial_size=[7, 7], window_spec=[8, 4, 16, 8]),
}
ALIASES = {"t": "tiny", "hiera_t": "tiny", "s": "small", "b+": "base_plus", "bplus": "base_plus",
           "hiera_b+": "base_plus", "l": "large", "hiera_l": "large"}


def model_config(size: str = "tiny", image_size: int = 512) -> dict:
    size = ALIASES.get(size, size)
    cfg = copy.deepcopy(_BASE)
    trunk = dict(TRUNKS[size])
    cfg["image_encoder"]["trunk"].update(trunk)
    e = trunk["embed_dim"]
    cfg["image_encoder"]["neck"]["backbone_channel_list"] = [8 * e, 4 * e, 2 * e, e]
    cfg["image_size"] = int(image_size)
    return cfg
