"""SAM2VideoPredictor -- the interactive video-inference surface the reference's evaluation
drives (reference sam2_video/eval/inference.py:361-577: `build_sam2_video_predictor`,
`init_state`, `add_new_points_or_box`, `add_new_mask`, `propagate_in_video` forward and in
reverse), running on the same libsam2hip kernels as the training step.

The reference imports this class from upstream `sam2` (inference.py:16, git HEAD, not vendored
in the reference and not installable offline); its behaviour is restated here from upstream's
published SAM2.1 algorithm (sam2/sam2_video_predictor.py):

  * per-object state (`output_dict_per_obj`, `temp_output_dict_per_obj`,
    `frames_tracked_per_obj`); clicks / masks go to a temporary dict and the memory encoder runs
    on them in `propagate_in_video_preflight` (binarised masks: `binarize_mask_from_pts_for_mem_enc`,
    which build_sam2_video_predictor turns on);
  * a frame that was not tracked yet is an initial conditioning frame (no memory, SAM-style);
    clicks on a tracked frame refine it, with the previous mask logits (clamped to +-32) as the
    dense mask prompt;
  * propagation yields (frame_idx, obj_ids, masks at the original video resolution);
    conditioning frames return their stored output, every other frame runs memory attention +
    SAM heads + memory encoder; the memory bank keeps every frame (selection by distance);
  * memory features are stored in bf16 (as upstream stores them), low-res mask logits in fp32;
  * optional hole filling of the low-res logits (`fill_hole_area`, 8 in build_sam2_video_predictor).

MI355X-first choices (not observable in the outputs): objects whose conditioning / tracked frame
sets agree are run as ONE batch through the kernels instead of one object at a time (each object
still reads only its own memory), and the image encoder runs on chunks of frames ahead of the
propagation and keeps their features resident in HBM.

Parity: with `binarize_mask_from_pts_for_mem_enc=False`, `fill_hole_area=0` and fp32 memory
storage, forward propagation from point prompts on frame 0 is the training step's forward in
eval mode, so tests pin it against the reference's golden per-frame logits
(tests/test_predictor_gpu.py).  Upstream-only behaviour (hole filling, binarisation, reverse
tracking, refinement clicks) has no reference fixture: parity unpinned, restated.
"""
from __future__ import annotations

import os
from collections import OrderedDict
from typing import Dict, List, Optional

import numpy as np
import torch

from .data.dataset import IMAGENET_MEAN, IMAGENET_STD
from .kernels import ops
from .model.modeling.sam2_base import NO_OBJ_SCORE


def _load_frames(video_path, image_size):
    """JPEG folder (frames named <int>.jpg, upstream's load_video_frames) or an array of frames
    [T, H, W, 3] uint8 -> (images [T, 3, S, S] fp32 ImageNet-normalised, video_H, video_W).
    A floating-point tensor [T, 3, S, S] is taken as already normalised model input (the
    training clips' `img_batch` layout; video resolution = S)."""
    from PIL import Image
    if isinstance(video_path, torch.Tensor) and video_path.is_floating_point():
        assert video_path.dim() == 4 and video_path.shape[1] == 3 and video_path.shape[-1] == image_size
        return video_path.float(), image_size, image_size
    if isinstance(video_path, (str, os.PathLike)):
        names = [p for p in os.listdir(video_path) if os.path.splitext(p)[-1].lower() in (".jpg", ".jpeg")]
        names.sort(key=lambda p: int(os.path.splitext(p)[0]))
        if not names:
            raise RuntimeError(f"no JPEG frames found in {video_path}")
        pil = [Image.open(os.path.join(video_path, n)).convert("RGB") for n in names]
    else:
        arr = video_path.numpy() if isinstance(video_path, torch.Tensor) else np.asarray(video_path)
        pil = [Image.fromarray(np.ascontiguousarray(f.astype(np.uint8))) for f in arr]
    W, H = pil[0].size
    imgs = np.stack([np.asarray(p.resize((image_size, image_size))) for p in pil])  # [T, S, S, 3]
    x = torch.from_numpy(imgs).permute(0, 3, 1, 2).float() / 255.0
    mean = torch.tensor(IMAGENET_MEAN).view(1, 3, 1, 1)
    std = torch.tensor(IMAGENET_STD).view(1, 3, 1, 1)
    return (x - mean) / std, H, W


def _connected_components(binary):
    """8-connected components -> (labels, per-pixel component area); host scipy on the low-res
    mask (upstream's get_connected_components contract)"""
    from scipy import ndimage
    lab, n = ndimage.label(binary, structure=np.ones((3, 3), dtype=np.int32))
    areas = np.bincount(lab.ravel(), minlength=n + 1)
    return lab, areas[lab]


def fill_holes_in_mask_scores(mask: torch.Tensor, max_area: int) -> torch.Tensor:
    """upstream sam2/utils/misc.py fill_holes_in_mask_scores: background components (score <= 0)
    of area <= max_area become 0.1, then foreground sprinkles (score > 0) of area <= max_area
    become -0.1.  mask [N, 1, h, w] fp32."""
    assert max_area > 0, "max_area must be positive"
    m = mask.detach().float().cpu().numpy()
    for i in range(m.shape[0]):
        lab, area = _connected_components(m[i, 0] <= 0)
        m[i, 0] = np.where((lab > 0) & (area <= max_area), 0.1, m[i, 0])
        lab, area = _connected_components(m[i, 0] > 0)
        m[i, 0] = np.where((lab > 0) & (area <= max_area), -0.1, m[i, 0])
    return torch.from_numpy(m).to(mask.device)


class SAM2VideoPredictor:
    """Wraps a loaded SAM2Model (every nn.Module attribute -- sam_mask_decoder, image_size,
    state_dict, ... -- is reachable on the predictor, as on upstream's SAM2Base subclass)."""

    def __init__(self, model, fill_hole_area: int = 0, non_overlap_masks: bool = False,
                 clear_non_cond_mem_around_input: bool = False, add_all_frames_to_correct_as_cond: bool = False,
                 binarize_mask_from_pts_for_mem_enc: bool = True, maskmem_storage_dtype=torch.bfloat16,
                 frame_chunk: int = 8):
        if model.arena is None:
            raise RuntimeError("call SAM2Model.load(device) before building a predictor")
        object.__setattr__(self, "model", model)
        self.fill_hole_area = fill_hole_area
        self.non_overlap_masks = non_overlap_masks
        self.clear_non_cond_mem_around_input = clear_non_cond_mem_around_input
        self.add_all_frames_to_correct_as_cond = add_all_frames_to_correct_as_cond
        self.binarize_mask_from_pts_for_mem_enc = binarize_mask_from_pts_for_mem_enc
        self.maskmem_storage_dtype = maskmem_storage_dtype
        self.frame_chunk = max(1, int(frame_chunk))
        model.eval()

    def __getattr__(self, name):
        return getattr(self.model, name)

    def load_state_dict(self, state_dict, strict: bool = True):
        """into the parameter arena (the bf16 compute shadow is refreshed)"""
        with torch.no_grad():
            own = self.model.state_dict()
            missing = [k for k in own if k not in state_dict]
            unexpected = [k for k in state_dict if k not in own]
            if strict and (missing or unexpected):
                raise RuntimeError(f"state_dict mismatch: missing {missing[:3]}, unexpected {unexpected[:3]}")
            for k, v in state_dict.items():
                if k in own:
                    own[k].copy_(v.to(own[k].device, own[k].dtype))
        self.model.arena.refresh_shadow()
        return missing, unexpected

    # ------------------------------------------------------------------ state
    @torch.no_grad()
    def init_state(self, video_path, offload_video_to_cpu: bool = False, offload_state_to_cpu: bool = False,
                   async_loading_frames: bool = False):
        if offload_state_to_cpu:
            raise NotImplementedError("the bank stays in HBM (288 GB per MI355X)")
        m = self.model
        device = m.arena.device
        # weights may have been loaded into a submodule in place (the reference's
        # _load_finetuned_weights_into_predictor): refresh the bf16 compute shadow
        m.arena.refresh_shadow()
        images, H, W = _load_frames(video_path, m.image_size)
        state = {
            "images": images if offload_video_to_cpu else images.to(device),
            "num_frames": images.shape[0], "video_height": H, "video_width": W, "device": device,
            "storage_device": device, "point_inputs_per_obj": {}, "mask_inputs_per_obj": {},
            "cached_features": {}, "constants": {}, "obj_id_to_idx": OrderedDict(),
            "obj_idx_to_id": OrderedDict(), "obj_ids": [], "output_dict_per_obj": {},
            "temp_output_dict_per_obj": {}, "frames_tracked_per_obj": {}, "tracking_has_started": False,
        }
        self._get_image_feature(state, 0)  # warm up the backbone, as upstream does
        return state

    def reset_state(self, inference_state):
        s = inference_state
        s["point_inputs_per_obj"].clear()
        s["mask_inputs_per_obj"].clear()
        s["constants"].clear()
        s["obj_id_to_idx"].clear()
        s["obj_idx_to_id"].clear()
        s["obj_ids"].clear()
        s["output_dict_per_obj"].clear()
        s["temp_output_dict_per_obj"].clear()
        s["frames_tracked_per_obj"].clear()
        s["tracking_has_started"] = False

    def _obj_id_to_idx(self, s, obj_id):
        idx = s["obj_id_to_idx"].get(obj_id)
        if idx is not None:
            return idx
        if s["tracking_has_started"]:
            raise RuntimeError(f"Cannot add new object id {obj_id} after tracking starts. All existing object ids: "
                               f"{s['obj_ids']}. Please call 'reset_state' to restart from scratch.")
        idx = len(s["obj_id_to_idx"])
        s["obj_id_to_idx"][obj_id] = idx
        s["obj_idx_to_id"][idx] = obj_id
        s["obj_ids"] = list(s["obj_id_to_idx"])
        s["point_inputs_per_obj"][idx] = {}
        s["mask_inputs_per_obj"][idx] = {}
        s["output_dict_per_obj"][idx] = {"cond_frame_outputs": {}, "non_cond_frame_outputs": {}}
        s["temp_output_dict_per_obj"][idx] = {"cond_frame_outputs": {}, "non_cond_frame_outputs": {}}
        s["frames_tracked_per_obj"][idx] = {}
        return idx

    # --------------------------------------------------------------- features
    def _get_image_feature(self, s, frame_idx, direction: int = 1):
        """(feat [L, C], pos [L, C], s0 [1, 4h, 4w, C0], s1 [1, 2h, 2w, C1]) of a frame; the
        backbone runs on a chunk of frames in the tracking direction and keeps them resident"""
        cache = s["cached_features"]
        if frame_idx not in cache:
            T = s["num_frames"]
            lo, hi = (frame_idx, min(T, frame_idx + self.frame_chunk)) if direction >= 0 else \
                (max(0, frame_idx - self.frame_chunk + 1), frame_idx + 1)
            todo = [t for t in range(lo, hi) if t not in cache]
            m = self.model
            img = s["images"][todo[0]:todo[-1] + 1].to(s["device"], non_blocking=True)
            bo = m.forward_image(img)
            fpn, pos = bo["backbone_fpn"], bo["vision_pos_enc"][-1]
            h = m.sam_image_embedding_size
            feats = fpn[-1].reshape(len(todo), h * h, -1)
            for i, t in enumerate(range(todo[0], todo[-1] + 1)):
                cache[t] = (feats[i], pos, fpn[0][i:i + 1], fpn[1][i:i + 1])
        return cache[frame_idx]

    # ------------------------------------------------------------------ prompts
    @torch.no_grad()
    def add_new_points_or_box(self, inference_state, frame_idx, obj_id, points=None, labels=None,
                              clear_old_points=True, normalize_coords=True, box=None):
        s = inference_state
        obj_idx = self._obj_id_to_idx(s, obj_id)
        if (points is not None) != (labels is not None):
            raise ValueError("points and labels must be provided together")
        if points is None and box is None:
            raise ValueError("at least one of points or box must be provided as input")
        points = torch.zeros(0, 2) if points is None else torch.as_tensor(points, dtype=torch.float32).cpu()
        labels = torch.zeros(0, dtype=torch.int32) if labels is None else \
            torch.as_tensor(labels, dtype=torch.int32).cpu()
        if points.dim() == 2:
            points = points.unsqueeze(0)
        if labels.dim() == 1:
            labels = labels.unsqueeze(0)
        if box is not None:
            if not clear_old_points:
                raise ValueError("cannot add box without clearing old points, since box prompt must be provided "
                                 "before any point prompt (please use clear_old_points=True instead)")
            box = torch.as_tensor(box, dtype=torch.float32).cpu().reshape(1, 2, 2)
            points = torch.cat([box, points], dim=1)
            labels = torch.cat([torch.tensor([[2, 3]], dtype=torch.int32), labels], dim=1)
        if normalize_coords:
            points = points / torch.tensor([s["video_width"], s["video_height"]], dtype=torch.float32)
        points = points * self.model.image_size
        old = s["point_inputs_per_obj"][obj_idx].get(frame_idx) if not clear_old_points else None
        if old is not None:
            points = torch.cat([old["point_coords"], points], dim=1)
            labels = torch.cat([old["point_labels"], labels], dim=1)
        point_inputs = {"point_coords": points, "point_labels": labels}
        s["point_inputs_per_obj"][obj_idx][frame_idx] = point_inputs
        s["mask_inputs_per_obj"][obj_idx].pop(frame_idx, None)
        return self._add_prompt(s, obj_idx, frame_idx, point_inputs=point_inputs)

    @torch.no_grad()
    def add_new_mask(self, inference_state, frame_idx, obj_id, mask):
        s = inference_state
        obj_idx = self._obj_id_to_idx(s, obj_id)
        mask = torch.as_tensor(mask).cpu()
        assert mask.dim() == 2
        S = self.model.image_size
        m = mask[None, None].float()
        if m.shape[-2:] != (S, S):
            m = torch.nn.functional.interpolate(m, size=(S, S), align_corners=False, mode="bilinear",
                                                antialias=True)
            m = (m >= 0.5).float()
        s["mask_inputs_per_obj"][obj_idx][frame_idx] = m
        s["point_inputs_per_obj"][obj_idx].pop(frame_idx, None)
        return self._add_prompt(s, obj_idx, frame_idx, mask_inputs=m)

    def _add_prompt(self, s, obj_idx, frame_idx, point_inputs=None, mask_inputs=None):
        tracked = s["frames_tracked_per_obj"][obj_idx]
        is_init_cond_frame = frame_idx not in tracked
        reverse = False if is_init_cond_frame else tracked[frame_idx]["reverse"]
        is_cond = is_init_cond_frame or self.add_all_frames_to_correct_as_cond
        key = "cond_frame_outputs" if is_cond else "non_cond_frame_outputs"
        out_d, temp_d = s["output_dict_per_obj"][obj_idx], s["temp_output_dict_per_obj"][obj_idx]
        prev_logits = None
        if point_inputs is not None:
            prev = temp_d[key].get(frame_idx) or out_d["cond_frame_outputs"].get(frame_idx) or \
                out_d["non_cond_frame_outputs"].get(frame_idx)
            if prev is not None and prev["pred_masks"] is not None:
                prev_logits = prev["pred_masks"].clamp(-32.0, 32.0)
        outs = self._run_single_frame_inference(s, [obj_idx], frame_idx, is_init_cond_frame, point_inputs,
                                                mask_inputs, reverse, run_mem_encoder=False,
                                                prev_sam_mask_logits=prev_logits)
        temp_d[key][frame_idx] = outs[0]
        masks = self._consolidate(s, frame_idx, is_cond)
        return frame_idx, list(s["obj_ids"]), self._video_res(s, masks)

    def _consolidate(self, s, frame_idx, is_cond):
        """low-res logits of every object at a frame (temporary output first, then the bank;
        NO_OBJ_SCORE where an object has none) -> [N, 1, 4h, 4w]"""
        key = "cond_frame_outputs" if is_cond else "non_cond_frame_outputs"
        h4 = 4 * self.model.sam_image_embedding_size
        res = []
        for i in range(len(s["obj_ids"])):
            out = (s["temp_output_dict_per_obj"][i][key].get(frame_idx)
                   or s["output_dict_per_obj"][i]["cond_frame_outputs"].get(frame_idx)
                   or s["output_dict_per_obj"][i]["non_cond_frame_outputs"].get(frame_idx))
            res.append(out["pred_masks"] if out is not None else
                       torch.full((1, 1, h4, h4), NO_OBJ_SCORE, device=s["device"]))
        return torch.cat(res, dim=0)

    def _video_res(self, s, masks):
        """[N, 1, h, w] low-res logits -> [N, 1, video_H, video_W] (bilinear, align_corners False)"""
        N, _, h, w = masks.shape
        out = ops.bilinear(masks.reshape(N, h, w).contiguous(), s["video_height"], s["video_width"])
        out = out.view(N, 1, s["video_height"], s["video_width"])
        if self.non_overlap_masks and N > 1:
            out = self._apply_non_overlapping_constraints(out)
        return out

    @staticmethod
    def _apply_non_overlapping_constraints(pred_masks):
        """upstream sam2_base._apply_non_overlapping_constraints: keep only the highest-scoring
        object per pixel; the others are clamped to <= -10"""
        keep = pred_masks.argmax(dim=0, keepdim=True) == torch.arange(pred_masks.shape[0],
                                                                       device=pred_masks.device)[:, None, None, None]
        return torch.where(keep, pred_masks, torch.clamp(pred_masks, max=-10.0))

    # --------------------------------------------------------------- inference
    def _bank_view(self, s, obj_idxs):
        """the objects' bank entries concatenated over objects (they share frame sets)"""
        d0 = s["output_dict_per_obj"][obj_idxs[0]]
        view = {"cond_frame_outputs": {}, "non_cond_frame_outputs": {}}
        for key in view:
            for t in d0[key]:
                es = [s["output_dict_per_obj"][i][key][t] for i in obj_idxs]
                if len(es) == 1:
                    e = es[0]
                    view[key][t] = {"maskmem_features": e["maskmem_features"], "maskmem_pos_enc": e["maskmem_pos_enc"],
                                    "obj_ptr": e["obj_ptr"]}
                else:
                    view[key][t] = {"maskmem_features": torch.cat([e["maskmem_features"] for e in es]),
                                    "maskmem_pos_enc": es[0]["maskmem_pos_enc"],
                                    "obj_ptr": torch.cat([e["obj_ptr"] for e in es])}
        return view

    def _mem_dtype(self, x):
        """bank storage: bf16 as upstream stores it, read back in the compute dtype"""
        if self.maskmem_storage_dtype is None or x.dtype == self.maskmem_storage_dtype:
            return x
        return ops.cast(ops.cast(x.contiguous(), self.maskmem_storage_dtype), x.dtype)

    def _run_single_frame_inference(self, s, obj_idxs, frame_idx, is_init_cond_frame, point_inputs, mask_inputs,
                                    reverse, run_mem_encoder, prev_sam_mask_logits=None):
        """track_step of a batch of objects sharing their frame sets -> one output dict per object"""
        m = self.model
        O = len(obj_idxs)
        feat, pos, s0, s1 = self._get_image_feature(s, frame_idx, -1 if reverse else 1)
        h = m.sam_image_embedding_size
        dev = s["device"]
        pe1, lab1 = self._pad_prompt(s, O)
        if mask_inputs is not None:
            mk = mask_inputs.reshape(O, m.image_size, m.image_size).to(dev)
            score = ((mask_inputs.reshape(O, -1).amax(dim=1) > 0).float() * 20.0 - 10.0).to(dev)
            m._mask_pad_prompt = (pe1, lab1)
            low, high, _, ptr, score = m._use_mask_as_output(feat, mk, score, (s0, s1), O)
        else:
            if is_init_cond_frame:
                pix = m._prepare_memory_conditioned_features(frame_idx, True, feat, pos, s["num_frames"], None, O)
            else:
                bank = self._bank_view(s, obj_idxs)
                pix = m._prepare_memory_conditioned_features(frame_idx, False, feat, pos, s["num_frames"], bank, O,
                                                             track_in_reverse=reverse)
            if point_inputs is not None:
                pe, lab = m.sam_prompt_encoder.host_points(point_inputs["point_coords"], point_inputs["point_labels"],
                                                           pad=True)
                prompt = (pe.to(dev), lab.to(dev))
            else:
                prompt = (pe1, lab1)
            dense = None
            if prev_sam_mask_logits is not None:
                dense = m.sam_prompt_encoder.dense_from_mask(
                    prev_sam_mask_logits.reshape(O, 4 * h, 4 * h, 1).contiguous(), m.compute_dtype)
            low, high, _, ptr, score = m._forward_sam_heads(pix, prompt, (s0, s1), O, dense=dense)
        low = low.view(O, 1, 4 * h, 4 * h)
        mfeat = mpos = None
        if run_mem_encoder:
            mfeat, mpos = self._encode(feat, high, score, O, point_inputs is not None)
        if self.fill_hole_area > 0:
            low = fill_holes_in_mask_scores(low, self.fill_hole_area)
        outs = []
        for i in range(O):
            outs.append({"maskmem_features": None if mfeat is None else mfeat[i:i + 1],
                         "maskmem_pos_enc": mpos, "pred_masks": low[i:i + 1], "obj_ptr": ptr[i:i + 1],
                         "object_score_logits": score.reshape(O, 1)[i:i + 1]})
        return outs

    def _pad_prompt(self, s, O):
        c = s["constants"].get(("pad", O))
        if c is None:
            pe1, lab1 = self.model.sam_prompt_encoder.host_points(torch.zeros(O, 1, 2),
                                                                  -torch.ones(O, 1, dtype=torch.int32), pad=True)
            c = s["constants"][("pad", O)] = (pe1.to(s["device"]), lab1.to(s["device"]))
        return c

    def _encode(self, feat, high, score, O, is_mask_from_pts):
        """_encode_new_memory with upstream's eval-time binarisation of user-interacted frames"""
        m = self.model
        if is_mask_from_pts and self.binarize_mask_from_pts_for_mem_enc:
            # binarised masks (pred > 0) enter the encoder as 0/1: logits of +-1e4 give exactly that
            # through the fused sigmoid(x) * scale + bias of the first down-sampling stage
            high = torch.where(high > 0, 1e4, -1e4).to(high.dtype)
        mfeat, mpos = m._encode_new_memory(feat, high, score, O)
        return self._mem_dtype(mfeat.reshape(O, -1, m.mem_dim)), mpos

    # ------------------------------------------------------------- propagation
    @torch.no_grad()
    def propagate_in_video_preflight(self, inference_state):
        s = inference_state
        s["tracking_has_started"] = True
        n = len(s["obj_ids"])
        m = self.model
        S = m.image_size
        for i in range(n):
            out_d, temp_d = s["output_dict_per_obj"][i], s["temp_output_dict_per_obj"][i]
            for key in ("non_cond_frame_outputs", "cond_frame_outputs"):
                for t, out in temp_d[key].items():
                    if out["maskmem_features"] is None:
                        feat = self._get_image_feature(s, t)[0]
                        pm = out["pred_masks"]
                        high = ops.bilinear(pm.reshape(1, pm.shape[-2], pm.shape[-1]).contiguous(), S, S)
                        mf, mp = self._encode(feat, high, out["object_score_logits"].reshape(-1).contiguous(), 1, True)
                        out["maskmem_features"], out["maskmem_pos_enc"] = mf, mp
                    out_d[key][t] = out
                    if self.clear_non_cond_mem_around_input:
                        r = m.memory_temporal_stride_for_eval * m.num_maskmem
                        for tt in range(t - r, t + r + 1):
                            out_d["non_cond_frame_outputs"].pop(tt, None)
                temp_d[key].clear()
            if not out_d["cond_frame_outputs"]:
                raise RuntimeError(f"No input points or masks are provided for object id {s['obj_idx_to_id'][i]}; "
                                   "please add inputs first.")
            for t in out_d["cond_frame_outputs"]:
                out_d["non_cond_frame_outputs"].pop(t, None)

    @torch.no_grad()
    def propagate_in_video(self, inference_state, start_frame_idx=None, max_frame_num_to_track=None,
                           reverse=False):
        s = inference_state
        self.propagate_in_video_preflight(s)
        obj_ids = s["obj_ids"]
        n = len(obj_ids)
        T = s["num_frames"]
        if start_frame_idx is None:
            start_frame_idx = min(t for d in s["output_dict_per_obj"].values() for t in d["cond_frame_outputs"])
        if max_frame_num_to_track is None:
            max_frame_num_to_track = T
        if reverse:
            end = max(start_frame_idx - max_frame_num_to_track, 0)
            order = range(start_frame_idx, end - 1, -1) if start_frame_idx > 0 else []
        else:
            end = min(start_frame_idx + max_frame_num_to_track, T - 1)
            order = range(start_frame_idx, end + 1)
        for t in order:
            per_obj: List[Optional[torch.Tensor]] = [None] * n
            todo = []
            for i in range(n):
                d = s["output_dict_per_obj"][i]
                if t in d["cond_frame_outputs"]:
                    per_obj[i] = d["cond_frame_outputs"][t]["pred_masks"]
                    if self.clear_non_cond_mem_around_input:
                        r = self.model.memory_temporal_stride_for_eval * self.model.num_maskmem
                        for tt in range(t - r, t + r + 1):
                            d["non_cond_frame_outputs"].pop(tt, None)
                else:
                    todo.append(i)
            for group in self._groups(s, todo):
                outs = self._run_single_frame_inference(s, group, t, False, None, None, reverse, run_mem_encoder=True)
                for i, out in zip(group, outs):
                    s["output_dict_per_obj"][i]["non_cond_frame_outputs"][t] = out
                    per_obj[i] = out["pred_masks"]
            for i in range(n):
                s["frames_tracked_per_obj"][i][t] = {"reverse": reverse}
            masks = torch.cat(per_obj, dim=0) if n > 1 else per_obj[0]
            yield t, obj_ids, self._video_res(s, masks)

    @staticmethod
    def _groups(s, obj_idxs) -> List[List[int]]:
        """objects whose bank holds the same frames run as one batch"""
        groups: Dict[tuple, List[int]] = OrderedDict()
        for i in obj_idxs:
            d = s["output_dict_per_obj"][i]
            key = (tuple(sorted(d["cond_frame_outputs"])), tuple(sorted(d["non_cond_frame_outputs"])))
            groups.setdefault(key, []).append(i)
        return list(groups.values())

    # --------------------------------------------------------------- editing
    @torch.no_grad()
    def clear_all_prompts_in_frame(self, inference_state, frame_idx, obj_id, need_output=True):
        s = inference_state
        i = self._obj_id_to_idx(s, obj_id)
        s["point_inputs_per_obj"][i].pop(frame_idx, None)
        s["mask_inputs_per_obj"][i].pop(frame_idx, None)
        temp = s["temp_output_dict_per_obj"][i]
        temp["cond_frame_outputs"].pop(frame_idx, None)
        temp["non_cond_frame_outputs"].pop(frame_idx, None)
        d = s["output_dict_per_obj"][i]
        out = d["cond_frame_outputs"].pop(frame_idx, None)
        if out is not None:
            d["non_cond_frame_outputs"][frame_idx] = out
            s["frames_tracked_per_obj"][i].pop(frame_idx, None)
        if not need_output:
            return
        masks = self._consolidate(s, frame_idx, is_cond=True)
        return frame_idx, list(s["obj_ids"]), self._video_res(s, masks)

    @torch.no_grad()
    def remove_object(self, inference_state, obj_id, strict=False, need_output=True):
        s = inference_state
        if obj_id not in s["obj_id_to_idx"]:
            if strict:
                raise RuntimeError(f"Cannot remove object id {obj_id} as it doesn't exist. "
                                   f"All existing object ids: {s['obj_ids']}.")
            return list(s["obj_ids"]), []
        old = s["obj_id_to_idx"][obj_id]
        remain = [i for i in range(len(s["obj_ids"])) if i != old]
        for k in ("point_inputs_per_obj", "mask_inputs_per_obj", "output_dict_per_obj", "temp_output_dict_per_obj",
                  "frames_tracked_per_obj"):
            s[k] = {new: s[k][i] for new, i in enumerate(remain)}
        ids = [s["obj_idx_to_id"][i] for i in remain]
        s["obj_id_to_idx"] = OrderedDict((oid, n) for n, oid in enumerate(ids))
        s["obj_idx_to_id"] = OrderedDict((n, oid) for n, oid in enumerate(ids))
        s["obj_ids"] = ids
        if not need_output or not ids:
            return list(ids), []
        frames = sorted({t for d in s["output_dict_per_obj"].values() for t in d["cond_frame_outputs"]})
        return list(ids), [(t, self._video_res(s, self._consolidate(s, t, is_cond=True))) for t in frames]


def build_sam2_video_predictor(config_file, ckpt_path=None, device="cuda", mode="eval", hydra_overrides_extra=(),
                               apply_postprocessing=True, vos_optimized=False, compute_dtype="bf16", image_size=None,
                               **kwargs):
    """upstream sam2.build_sam.build_sam2_video_predictor: the SAM2.1 model of `config_file`
    (named sizes, upstream config names or a YAML path, model/build.py) with `ckpt_path`
    weights (deterministic synthetic weights when absent, as everywhere offline), as a
    predictor with upstream's post-processing (binarised user masks into memory, hole filling
    of area <= 8)."""
    from .model.sam2model import SAM2Model
    model = SAM2Model(ckpt_path, config_file, trainable_modules=[], compute_dtype=compute_dtype,
                      image_size=image_size, **kwargs)
    model.load(device)
    if mode == "eval":
        model.eval()
    return SAM2VideoPredictor(model, fill_hole_area=8 if apply_postprocessing else 0,
                              binarize_mask_from_pts_for_mem_enc=True)
