"""SAM2Model -- drop-in for sam2_video.model.sam2model.SAM2Model (reference
sam2_video/model/sam2model.py:28-616): same constructor, same
forward(BatchedVideoDatapoint) -> (per-frame category-level outputs, obj_to_cat),
same state_dict keys as upstream SAM2 (checkpoints load), same freezing
semantics.  The heavy lifting runs in libsam2hip on the GPU.

Differences that are not observable in the outputs:
  * the reference builds an upstream model and grafts its attributes onto a
    SAM2Base (sam2model.py:80-105); this build instantiates its own modules
    directly from the same config;
  * parameters live in a flat device arena (kernels/arena.py) after `load(device)`;
  * the memory encoder runs without an autograd tape (its outputs are detached
    into the memory bank in the reference, so it never receives a gradient).
"""
from __future__ import annotations

import os
from collections import OrderedDict
from typing import Any, Dict, List, Optional, Tuple

import torch
from torch import nn

from .. import utils
from ..data.data_utils import BatchedVideoDatapoint
from ..kernels import fp8, ops
from ..kernels.arena import ParamArena
from ..utils.init import synth_tensor
from ..utils.masks import merge_object_results_to_category
from .build import instantiate, load_model_config
from .modeling.sam2_base import SAM2Base

DTYPES = {"bf16": torch.bfloat16, "bfloat16": torch.bfloat16, "fp32": torch.float32, "float32": torch.float32,
          torch.bfloat16: torch.bfloat16, torch.float32: torch.float32,
          # MX-fp8 projections / FFN (kernels/fp8.py) over bf16 activations and shadow weights
          "fp8": torch.bfloat16, "mxfp8": torch.bfloat16}


class SAM2Model(SAM2Base):
    def __init__(self, checkpoint_path: Optional[str], config_path: str, fintuned_model_path: Optional[str] = None,
                 trainable_modules: Optional[List[str]] = None, device: str = "cuda", prompt_type: str = "point",
                 forward_backbone_per_frame_for_eval: bool = False, num_pos_points: int = 1,
                 num_neg_points: int = 0, include_center: bool = True, use_activation_checkpoint: bool = False,
                 random_init_memory_modules: bool = False, compute_dtype="bf16", image_size: Optional[int] = None,
                 init_seed: int = 0):
        self.checkpoint_path = checkpoint_path
        self.config_path = config_path
        self.prompt_type = prompt_type
        assert prompt_type in ["point", "box", "mask"], f"prompt_type must be one of point/box/mask, got {prompt_type}"
        self.forward_backbone_per_frame_for_eval = forward_backbone_per_frame_for_eval
        self.num_pos_points = num_pos_points
        self.num_neg_points = num_neg_points
        self.include_center = include_center
        self.fintuned_model_path = fintuned_model_path
        cfg = load_model_config(config_path, image_size)
        kw = {k: instantiate(v) for k, v in cfg.items() if k != "_target_"}
        super().__init__(use_activation_checkpoint=use_activation_checkpoint, **kw)
        if prompt_type == "mask" and not self.use_mask_input_as_output_without_sam:
            raise NotImplementedError("mask prompts through the SAM heads (use_mask_input_as_output_without_sam "
                                      "False) are not built; the SAM2.1 configs set it True")
        self.compute_dtype = DTYPES[compute_dtype]
        self.fp8 = compute_dtype in ("fp8", "mxfp8")
        # training steps run the tracking loop's backward frame-batched (model/tracking.py);
        # False = per-frame autograd (the reference's graph shape; A/B and tests)
        self.frame_batched = os.environ.get("S2H_FRAME_BATCHED", "1") != "0"
        self.arena: Optional[ParamArena] = None
        self._load_weights(checkpoint_path, init_seed)
        if fintuned_model_path is not None:
            self._load_finetuned(fintuned_model_path)
        if random_init_memory_modules:
            self._randomly_initialize_memory_modules(init_seed + 1)
        self._setup_trainable_modules(trainable_modules or ["memory_attention", "memory_encoder"])

    # ----------------------------------------------------------- weights
    def _load_weights(self, checkpoint_path, seed):
        """A SAM2.1 checkpoint (`{"model": state_dict}`, as upstream build_sam2 loads it, strict) or,
        with checkpoint_path None only, deterministic synthetic weights keyed by parameter name (no
        checkpoints exist offline).  A path that does not exist raises, as upstream build_sam2 does
        (reference sam2model.py:80-82) -- a mistyped path never trains from random weights."""
        sd = self.state_dict()
        if checkpoint_path is None:
            self.load_state_dict({k: synth_tensor(k, v.shape, seed) for k, v in sd.items()}, strict=True)
            return
        if not os.path.isfile(str(checkpoint_path)):
            raise FileNotFoundError(f"SAM2 checkpoint not found: {checkpoint_path} (pass checkpoint_path=None "
                                    "for deterministic synthetic weights)")
        ck = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
        if isinstance(ck, dict) and "model" in ck:
            ck = ck["model"]
        self.load_state_dict(ck, strict=True)

    @staticmethod
    def strip_lightning_prefix(ck):
        """Lightning .ckpt -> model state_dict: the `state_dict` entry with the `model.` prefix of
        SAM2LightningModule.model removed (reference train.py:146-157)"""
        sd = ck["state_dict"] if isinstance(ck, dict) and "state_dict" in ck else ck
        if any(k.startswith("model.") for k in sd):
            sd = {k[len("model."):]: v for k, v in sd.items() if k.startswith("model.")}
        return sd

    def load_lightning_checkpoint(self, path, strict: bool = True):
        """weights of a Lightning checkpoint of SAM2LightningModule (Trainer.save_checkpoint or the
        reference's ModelCheckpoint files); re-run load(device) afterwards if the arena exists"""
        ck = torch.load(path, map_location="cpu", weights_only=True)
        sd = self.strip_lightning_prefix(ck)
        if self.arena is not None:  # parameters are arena views: copy in place
            with torch.no_grad():
                own = self.state_dict()
                missing = [k for k in own if k not in sd]
                if strict and missing:
                    raise KeyError(f"checkpoint misses {len(missing)} keys, e.g. {missing[:3]}")
                for k, v in sd.items():
                    if k in own:
                        own[k].copy_(v.to(own[k].device, own[k].dtype))
            self.arena.refresh_shadow()
            return self
        self.load_state_dict(sd, strict=strict)
        return self

    def _load_finetuned(self, path):
        """sam2model.py:109-126 (an "all" path holds a full state dict; a Lightning .ckpt is
        unwrapped as train.py:146-157 does)"""
        if path.count("all") > 0 or path.endswith(".ckpt"):
            sd = torch.load(path, map_location="cpu", weights_only=True)
            sd = sd if isinstance(sd, (dict, OrderedDict)) else sd.state_dict()
            self.load_state_dict(self.strip_lightning_prefix(sd), strict=False)
        else:
            self.sam_mask_decoder.load_state_dict(torch.load(path, map_location="cpu", weights_only=True), strict=True)
            pe_path = path.replace(".torch", "_prompt_encoder.torch")
            if os.path.exists(pe_path):
                self.sam_prompt_encoder.load_state_dict(torch.load(pe_path, map_location="cpu", weights_only=True),
                                                        strict=True)

    def _randomly_initialize_memory_modules(self, seed):
        for name in ("memory_attention", "memory_encoder"):
            mod = getattr(self, name)
            for n, p in mod.named_parameters():
                p.data.copy_(synth_tensor(f"{name}.{n}", p.shape, seed))

    def _get_module_mapping(self) -> Dict[str, nn.Module]:
        """sam2model.py:550-565"""
        return {"image_encoder": self.image_encoder, "memory_attention": self.memory_attention,
                "memory_encoder": self.memory_encoder, "prompt_encoder": self.sam_prompt_encoder,
                "mask_decoder": self.sam_mask_decoder, "obj_ptr_proj": self.obj_ptr_proj,
                "obj_ptr_tpos_proj": self.obj_ptr_tpos_proj}

    def _setup_trainable_modules(self, trainable_modules: List[str]) -> None:
        self.trainable_modules = list(trainable_modules)
        utils.setup_trainable_modules(self, self._get_module_mapping(), self.trainable_modules)

    def freeze_module(self, module_name):
        utils.freeze_module_by_name(self._get_module_mapping(), module_name)

    def unfreeze_module(self, module_name):
        utils.unfreeze_module_by_name(self._get_module_mapping(), module_name)

    def get_trainable_modules(self):
        return utils.get_trainable_module_names(self._get_module_mapping())

    def never_grad_parameter_names(self) -> List[str]:
        """Trainable parameters that the training step never reaches with a gradient (their
        .grad stays None in the reference, so AdamW skips them): the memory encoder and the
        object-pointer path (both detached into the bank, sam2model.py:340-358), the unused
        no-memory position encoding, the mask-prompt down-sampling convs (point/box prompts)
        and the object-score head (its logits only gate; pred_obj_scores=False in the loss)."""
        out = []
        for n, p in self.named_parameters():
            if not p.requires_grad:
                continue
            if self.prompt_type == "mask" and n == "no_mem_embed":
                out.append(n)  # the mask-prompt frame bypasses it (sam2_base.py:796-806); no other frame adds it
                continue
            if (n.startswith("memory_encoder.") or n in ("no_mem_pos_enc", "no_obj_ptr", "no_obj_embed_spatial")
                    or n.startswith("mask_downsample.") or n.startswith("sam_prompt_encoder.mask_downscaling.")
                    or n.startswith("sam_mask_decoder.pred_obj_score_head.") or n.startswith("obj_ptr_proj.")):
                out.append(n)
        return out

    def load(self, device: str = None) -> "SAM2Model":
        """Move to `device` and build the parameter arena (call again after re-freezing)."""
        device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        if device.type != "cuda":
            raise RuntimeError("SAM2Model runs on MI355X only (libsam2hip has no CPU path)")
        ops.wgrad_workspace(device)  # before any graph capture: the weight-gradient GEMM's partials
        for name, buf in self.named_buffers():
            mod = self.get_submodule(name.rsplit(".", 1)[0]) if "." in name else self
            setattr(mod, name.rsplit(".", 1)[-1], buf.to(device))
        never = set(self.never_grad_parameter_names())
        named = list(self.named_parameters())
        grad_names = [n for n, p in named if p.requires_grad and n not in never]
        groups = []
        for i, layer in enumerate(self.memory_attention.layers):
            groups += layer.arena_groups(f"memory_attention.layers.{i}")
        self.arena = ParamArena(named, grad_names, self.compute_dtype, device, groups=groups,
                                tail_rank=self._backbone_grad_rank())
        for m in self.modules():
            if hasattr(m, "bind_arena"):
                m.bind_arena(self.arena)
        if self.fp8:
            fp8.mark_modules(self)
        return self

    def _backbone_grad_rank(self):
        """Order of the arena's tail: the parameters whose gradients the backbone backward (phase 2
        of StepRunner's overlapped backward) completes, by the segment that completes them -- 0:
        conv_s0 / conv_s1 (applied to the backbone outputs in forward_image) and the FPN neck, then
        the Hiera stages last to first (1 = the last stage), patch / position embedding with the
        first stage.  Everything else (the tracking loop's parameters) precedes them."""
        ends = list(self.image_encoder.trunk.stage_ends)
        nst = len(ends)

        def rank(n):
            if n.startswith(("sam_mask_decoder.conv_s0.", "sam_mask_decoder.conv_s1.", "image_encoder.neck.")):
                return 0
            if n.startswith("image_encoder.trunk.blocks."):
                i = int(n.split(".")[3])
                return nst - next(s for s, e in enumerate(ends) if i <= e)
            if n.startswith("image_encoder."):
                return nst
            return None
        return rank

    def backbone_backward_segments(self, pending):
        """Phase 2 of the overlapped backward as segments: [(closure, rank)], run in order; after
        segment k every gradient of arena rank k (_backbone_grad_rank) is complete.  `pending` =
        [(backbone output, its gradient)] from phase 1.  Segment 0 runs the backward from the backbone
        outputs through conv_s0 / conv_s1 and the neck to the neck's inputs (aliases of the Hiera
        stage outputs, ImageEncoder.forward, so it stops there); segment k >= 1 runs stage nst - k
        from its output -- gradient = the neck's + the next stage's -- to the previous stage's output
        (the first stage to the image)."""
        enc = self.image_encoder
        stages = list(getattr(enc.trunk, "last_outputs", []))
        taps = list(getattr(enc, "last_neck_inputs", []))
        outs = [t for t, _ in pending]
        grads = [g for _, g in pending]
        nst = len(enc.trunk.stage_ends)
        if len(stages) != nst or len(taps) != nst or not all(x.requires_grad for x in stages):
            # frozen trunk: conv_s0 / conv_s1 (and the neck) only, one segment
            return [(lambda: torch.autograd.backward(outs, grads), 0)]
        gs = {}

        def seg0():
            for i, g in enumerate(torch.autograd.grad(outs, taps, grads, allow_unused=True)):
                gs[i] = g

        def seg_stage(i):
            def run():
                g = gs.pop(i, None)
                if g is None:
                    return
                if i == 0:
                    torch.autograd.backward([stages[0]], [g])
                    return
                (gprev,) = torch.autograd.grad([stages[i]], [stages[i - 1]], [g], allow_unused=True)
                if gprev is not None:
                    if gs.get(i - 1) is None:
                        gs[i - 1] = gprev
                    else:
                        ops.add(gs[i - 1], gprev, out=gs[i - 1])
            return run
        return [(seg0, 0)] + [(seg_stage(nst - k), k) for k in range(1, nst + 1)]

    def set_dropout(self, p: float):
        """override every dropout probability (p=0 gives the deterministic parity mode)"""
        for m in self.modules():
            if hasattr(m, "dropout_p"):
                m.dropout_p = p
            if hasattr(m, "dropout_value"):
                m.dropout_value = p

    def count_trainable_parameters(self) -> int:
        return utils.count_trainable_parameters(self)

    def count_total_parameters(self) -> int:
        return utils.count_total_parameters(self)

    def get_info(self) -> Dict[str, Any]:
        return utils.get_model_info(self, self.checkpoint_path, self.config_path, str(self.device))

    # ------------------------------------------------------------- forward
    def forward(self, input: BatchedVideoDatapoint) -> Tuple[List[Dict[str, Any]], List[int]]:
        """sam2model.py:153-179"""
        if self.arena is None:
            raise RuntimeError("call SAM2Model.load(device) before forward")
        if self.fp8:
            fp8.new_step()  # weights moved since the last forward: re-quantise on first use
        if self.training or not self.forward_backbone_per_frame_for_eval:
            backbone_out = self.forward_image(input.flat_img_batch)
            # the backbone outputs the tracking loop reads: the split point of a two-phase backward
            # (StepRunner overlaps the gradient all-reduce of everything after them with the image
            # encoder's backward)
            self.last_backbone_outputs = [t for t in backbone_out["backbone_fpn"] if t.requires_grad]
        else:
            # evaluation with forward_backbone_per_frame_for_eval (sam2model.py:164-169): each frame's
            # image features are computed when the tracking loop reaches it (forward_tracking)
            backbone_out = {"backbone_fpn": None, "vision_pos_enc": None}
            self.last_backbone_outputs = []
        backbone_out = self.prepare_prompt_inputs(backbone_out, input)
        stages = self.forward_tracking(backbone_out, input)
        out = merge_object_results_to_category(stages, backbone_out["obj_to_cat"], backbone_out["num_categories"])
        return out, backbone_out["obj_to_cat"]

    def host_prompt_plan(self, input, start_frame_idx=0) -> Dict[str, Any]:
        """Host half of prepare_prompt_inputs (sam2model.py:181-236): frame-0 category masks ->
        objects (opening + connected components) -> clicks -> point encodings.  Pure CPU work on
        the batch's host copy of frame 0 (no device sync); the captured (graphed) step takes its
        result as input."""
        hm = getattr(input, "host_masks0", None) if start_frame_idx == 0 else None
        masks0 = (hm if hm is not None else input.masks[start_frame_idx]).unsqueeze(1)
        center_only = (self.prompt_type == "point" and self.num_pos_points == 1 and self.num_neg_points == 0
                       and self.include_center)
        if center_only or self.prompt_type == "box":
            # the clicks need only the objects' moments: no object masks are materialised
            from ..utils.masks import object_moments
            from ..utils.prompts import box_prompt_from_moments, center_prompt_from_moments
            cats, st, _ = object_moments(masks0[:, 0])
            if len(cats) == 0:
                raise ValueError("cat_to_obj_mask: no objects found in category masks (fail-fast)")
            obj_to_cat, num_categories, O = cats.tolist(), int(masks0.shape[0]), len(cats)
            points, labels = (center_prompt_from_moments if center_only else box_prompt_from_moments)(st)
            return self._point_plan(start_frame_idx, obj_to_cat, num_categories, points, labels)
        obj_masks, obj_to_cat, num_categories = utils.cat_to_obj_mask(masks0)
        O = len(obj_to_cat)
        pe1, lab1 = self.sam_prompt_encoder.host_points(torch.zeros(O, 1, 2), -torch.ones(O, 1, dtype=torch.int32),
                                                        pad=True)
        if self.prompt_type == "mask":
            # the object masks are the prompt (sam2model.py:215-217); score = 20 * any(mask) - 10
            # (sam2_base.py:473-477) is a host-side fact of the prompt
            m = obj_masks.reshape(O, -1).float()
            score = (m.amax(dim=1) > 0).float() * 20.0 - 10.0
            return {"start_frame_idx": start_frame_idx, "obj_to_cat": obj_to_cat, "num_categories": num_categories,
                    "points": None, "labels": None, "mask": True,
                    "host": (obj_masks.reshape(O, *obj_masks.shape[-2:]).float(), score, pe1, lab1)}
        points, labels = utils.generate_point_prompt(obj_masks, num_pos_points=self.num_pos_points,
                                                     num_neg_points=self.num_neg_points,
                                                     include_center=self.include_center)
        return self._point_plan(start_frame_idx, obj_to_cat, num_categories, points, labels)

    def _point_plan(self, start_frame_idx, obj_to_cat, num_categories, points, labels):
        O = len(obj_to_cat)
        pe0, lab0 = self.sam_prompt_encoder.host_points(points, labels, pad=True)
        pe1, lab1 = self.sam_prompt_encoder.host_points(torch.zeros(O, 1, 2), -torch.ones(O, 1, dtype=torch.int32),
                                                        pad=True)
        return {"start_frame_idx": start_frame_idx, "obj_to_cat": obj_to_cat, "num_categories": num_categories,
                "points": points, "labels": labels, "host": (pe0, lab0, pe1, lab1)}

    @staticmethod
    def upload_prompt_plan(plan, device, out=None):
        """host tensors of a plan -> device (pinned staging, asynchronous); into `out` when given"""
        host = [t.pin_memory() for t in plan["host"]]
        if out is None:
            return tuple(t.to(device, non_blocking=True) for t in host)
        for d, h in zip(out, host):
            d.copy_(h, non_blocking=True)
        return out

    def prepare_prompt_inputs(self, backbone_out, input, start_frame_idx=0):
        """sam2model.py:181-236 -- frame-0 category masks -> objects -> clicks.  A batch that carries
        `prompt_plan` (with `dev` tensors already on the device: the graphed step) skips the host
        work; otherwise it runs here, while the GPU executes the already-queued image encoder."""
        plan = getattr(input, "prompt_plan", None)
        if plan is None or plan.get("start_frame_idx", 0) != start_frame_idx:
            plan = self.host_prompt_plan(input, start_frame_idx)
        dev = plan.get("dev") or self.upload_prompt_plan(plan, self.arena.device)
        backbone_out["num_frames"] = input.num_frames
        backbone_out["obj_to_cat"] = plan["obj_to_cat"]
        backbone_out["num_categories"] = plan["num_categories"]
        backbone_out["prompt_pad"] = (dev[2], dev[3])
        if plan.get("mask"):
            backbone_out["prompt_cond"] = None
            backbone_out["mask_cond"] = (dev[0], dev[1])
            backbone_out["point_inputs_per_frame"] = {}
            backbone_out["mask_inputs_per_frame"] = {start_frame_idx: dev[0]}
        else:
            backbone_out["prompt_cond"] = (dev[0], dev[1])
            backbone_out["point_inputs_per_frame"] = {start_frame_idx: {"point_coords": plan["points"],
                                                                        "point_labels": plan["labels"]}}
            backbone_out["mask_inputs_per_frame"] = {}
        return backbone_out

    def forward_tracking(self, backbone_out, input: BatchedVideoDatapoint, return_dict=False):
        """sam2model.py:266-401 -- sequential frames, detached memory bank pruned to the
        last num_maskmem-1 non-conditioning frames."""
        fpn = backbone_out["backbone_fpn"]
        T = backbone_out["num_frames"]
        h = w = self.sam_image_embedding_size
        if fpn is not None:
            feats = fpn[-1].reshape(T, h * w, -1)
            pos = backbone_out["vision_pos_enc"][-1]
            s0, s1 = fpn[0], fpn[1]
        else:  # per-frame backbone for evaluation (forward): frame t's features computed at frame t
            feats = s0 = s1 = pos = None
            imgs = input.flat_img_batch

        def frame_features(t):
            """(image embedding [h*w, C], its position table, high-res levels 0 / 1 of frame t)"""
            if fpn is not None:
                return feats[t], pos, s0[t:t + 1], s1[t:t + 1]
            out = self.forward_image(imgs[t:t + 1])
            f = out["backbone_fpn"]
            return f[-1].reshape(h * w, -1), out["vision_pos_enc"][-1], f[0], f[1]
        O = len(backbone_out["obj_to_cat"])
        output_dict = {"cond_frame_outputs": {}, "non_cond_frame_outputs": {}}
        frames = []
        mask_cond = backbone_out.get("mask_cond")
        if mask_cond is not None:
            if T <= 1 and self.training:
                raise NotImplementedError("mask prompts on single-frame training clips go through the SAM heads "
                                          "(sam2_base.py:796-800); not built")
            self._mask_pad_prompt = backbone_out["prompt_pad"]
        tracker = None
        if self.frame_batched and self.training and torch.is_grad_enabled() and not return_dict:
            from .tracking import FrameTracker
            pshape = [tuple(backbone_out["prompt_cond"][0].shape) if (t == 0 and mask_cond is None)
                      else tuple(backbone_out["prompt_pad"][0].shape) for t in range(T)]
            tracker = FrameTracker(self, T, O, feats, s0, s1, mask_cond is not None, pshape)
        for t in range(T):
            is_cond = t == 0
            feat_t, pos, s0_t, s1_t = frame_features(t)
            if is_cond and mask_cond is not None:
                low, high, ious, ptr, score = self._use_mask_as_output(feat_t, mask_cond[0], mask_cond[1],
                                                                       (s0_t, s1_t), O)
            elif tracker is not None:
                prompt = backbone_out["prompt_cond"] if is_cond else backbone_out["prompt_pad"]
                pix = tracker.memory_conditioned(t, feat_t.detach(), pos, output_dict)
                low, high, ious, ptr, score = tracker.sam_heads(t, pix, prompt, s0_t.detach(), s1_t.detach())
            else:
                pix = self._prepare_memory_conditioned_features(t, is_cond, feat_t, pos, T, output_dict, O)
                prompt = backbone_out["prompt_cond"] if is_cond else backbone_out["prompt_pad"]
                low, high, ious, ptr, score = self._forward_sam_heads(pix, prompt, (s0_t, s1_t), O)
            mfeat, mpos = self._encode_new_memory(feat_t, high, score, O)
            entry = {"maskmem_features": mfeat, "maskmem_pos_enc": mpos, "obj_ptr": ptr}
            if is_cond:
                output_dict["cond_frame_outputs"][t] = entry
            else:
                nc = output_dict["non_cond_frame_outputs"]
                nc[t] = entry
                while len(nc) > max(self.num_maskmem - 1, 0):
                    del nc[min(nc)]
            pin = backbone_out["point_inputs_per_frame"].get(t)
            low4 = low.view(O, 1, 4 * h, 4 * w)
            high4 = high.view(O, 1, self.image_size, self.image_size)
            minp = backbone_out["mask_inputs_per_frame"].get(t)
            frames.append({
                "point_inputs": pin, "mask_inputs": minp,
                "pred_masks": low4, "pred_masks_high_res": high4,
                "multistep_pred_masks": low4, "multistep_pred_masks_high_res": high4,
                "multistep_pred_multimasks": [low4], "multistep_pred_multimasks_high_res": [high4],
                "multistep_pred_ious": [ious], "multistep_point_inputs": [pin],
                "multistep_object_score_logits": [score],
            })
        if return_dict:
            return output_dict
        if tracker is not None:  # one autograd node for the whole loop (frame-batched backward)
            hi = tracker.finish()
            for t, fr in enumerate(frames):
                if t in hi:
                    high4 = hi[t][0].view(O, 1, self.image_size, self.image_size)
                    fr["pred_masks_high_res"] = fr["multistep_pred_masks_high_res"] = high4
                    fr["multistep_pred_multimasks_high_res"] = [high4]
                    fr["multistep_pred_ious"] = [hi[t][1]]
        return frames
