"""SAM2Base (reference sam2_video/model/modeling/sam2_base.py) -- the per-frame
machinery of the training step on MI355X.

Layout: every feature map is NHWC / token-major ([frames|objects, H*W, C]) in the
compute dtype; mask logits are fp32 (as the reference casts them, :391-399).
All arithmetic runs in libsam2hip; positional encodings, RoPE tables and the
object-pointer temporal encodings are cached host-evaluated constants.

Supported configuration: the SAM2.1 training setup of the reference YAML
(configs/sam2/sam2.1_hiera_t.yaml:87-121) -- high-res features, object pointers
with signed projected temporal encodings, object scores with fixed no-object
pointer, no-object spatial embedding, directly added no-memory embedding,
single-mask output.  Other flag values raise.
"""
from __future__ import annotations

import math
import warnings

import torch
from torch import nn

from ...kernels import functional as FN
from ...kernels import ops
from .layers import MLP, Conv2d, Linear
from .position_encoding import get_1d_sine_pe
from .sam.mask_decoder import MaskDecoder
from .sam.prompt_encoder import PromptEncoder
from .sam.transformer import TwoWayTransformer

NO_OBJ_SCORE = -1024.0  # sam2_base.py:18


class ActivationCheckpointNotice(UserWarning):
    """`use_activation_checkpoint=True` is accepted but does not recompute (see SAM2Base)"""


class SAM2Base(nn.Module):
    def __init__(self, image_encoder, memory_attention, memory_encoder, num_maskmem=7, image_size=512,
                 backbone_stride=16, sigmoid_scale_for_mem_enc=1.0, sigmoid_bias_for_mem_enc=0.0,
                 binarize_mask_from_pts_for_mem_enc=False, use_mask_input_as_output_without_sam=False,
                 max_cond_frames_in_attn=-1, directly_add_no_mem_embed=False, use_high_res_features_in_sam=False,
                 multimask_output_in_sam=False, multimask_min_pt_num=1, multimask_max_pt_num=1,
                 multimask_output_for_tracking=False, use_multimask_token_for_obj_ptr=False,
                 iou_prediction_use_sigmoid=False, memory_temporal_stride_for_eval=1,
                 non_overlap_masks_for_mem_enc=False, use_obj_ptrs_in_encoder=False, max_obj_ptrs_in_encoder=16,
                 add_tpos_enc_to_obj_ptrs=True, proj_tpos_enc_in_obj_ptrs=False,
                 use_signed_tpos_enc_to_obj_ptrs=False, only_obj_ptrs_in_the_past_for_eval=False,
                 pred_obj_scores=False, pred_obj_scores_mlp=False, fixed_no_obj_ptr=False, soft_no_obj_ptr=False,
                 use_mlp_for_obj_ptr_proj=False, no_obj_embed_spatial=False, sam_mask_decoder_extra_args=None,
                 compile_image_encoder=False, use_activation_checkpoint=False):
        super().__init__()
        self.image_encoder = image_encoder
        self.use_high_res_features_in_sam = use_high_res_features_in_sam
        self.num_feature_levels = 3 if use_high_res_features_in_sam else 1
        self.use_obj_ptrs_in_encoder = use_obj_ptrs_in_encoder
        self.max_obj_ptrs_in_encoder = max_obj_ptrs_in_encoder
        # The reference recomputes the memory attention / memory encoder / image encoder activations
        # in the backward when set (sam2_base.py:362,706,752): a memory-for-compute trade with
        # identical results.  Here every saved activation stays resident in HBM (a B+ 512^2 16-frame
        # step needs a few GB of the 288 GB per GPU), so the flag is accepted and only recorded.
        self.use_activation_checkpoint = bool(use_activation_checkpoint)
        if self.use_activation_checkpoint:
            warnings.warn("use_activation_checkpoint=True: accepted, no recompute -- activations stay resident in "
                          "HBM (results are identical; only peak memory differs from the reference)",
                          ActivationCheckpointNotice, stacklevel=2)
        if use_obj_ptrs_in_encoder:
            self.mask_downsample = Conv2d(1, 1, 4, 4)
        self.add_tpos_enc_to_obj_ptrs = add_tpos_enc_to_obj_ptrs
        self.proj_tpos_enc_in_obj_ptrs = proj_tpos_enc_in_obj_ptrs
        self.use_signed_tpos_enc_to_obj_ptrs = use_signed_tpos_enc_to_obj_ptrs
        self.only_obj_ptrs_in_the_past_for_eval = only_obj_ptrs_in_the_past_for_eval
        self.memory_attention = memory_attention
        self.hidden_dim = image_encoder.neck.d_model
        self.memory_encoder = memory_encoder
        self.mem_dim = self.hidden_dim
        if hasattr(self.memory_encoder, "out_proj") and hasattr(self.memory_encoder.out_proj, "weight"):
            self.mem_dim = self.memory_encoder.out_proj.weight.shape[0]
        self.num_maskmem = num_maskmem
        self.maskmem_tpos_enc = nn.Parameter(torch.zeros(num_maskmem, 1, 1, self.mem_dim))
        self.no_mem_embed = nn.Parameter(torch.zeros(1, 1, self.hidden_dim))
        self.no_mem_pos_enc = nn.Parameter(torch.zeros(1, 1, self.hidden_dim))
        self.directly_add_no_mem_embed = directly_add_no_mem_embed
        self.sigmoid_scale_for_mem_enc = sigmoid_scale_for_mem_enc
        self.sigmoid_bias_for_mem_enc = sigmoid_bias_for_mem_enc
        self.binarize_mask_from_pts_for_mem_enc = binarize_mask_from_pts_for_mem_enc
        self.non_overlap_masks_for_mem_enc = non_overlap_masks_for_mem_enc
        self.memory_temporal_stride_for_eval = memory_temporal_stride_for_eval
        self.use_mask_input_as_output_without_sam = use_mask_input_as_output_without_sam
        self.multimask_output_in_sam = multimask_output_in_sam
        self.multimask_min_pt_num = multimask_min_pt_num
        self.multimask_max_pt_num = multimask_max_pt_num
        self.multimask_output_for_tracking = multimask_output_for_tracking
        self.use_multimask_token_for_obj_ptr = use_multimask_token_for_obj_ptr
        self.iou_prediction_use_sigmoid = iou_prediction_use_sigmoid
        self.image_size = image_size
        self.backbone_stride = backbone_stride
        self.sam_mask_decoder_extra_args = sam_mask_decoder_extra_args
        self.pred_obj_scores = pred_obj_scores
        self.pred_obj_scores_mlp = pred_obj_scores_mlp
        self.fixed_no_obj_ptr = fixed_no_obj_ptr
        self.soft_no_obj_ptr = soft_no_obj_ptr
        if self.pred_obj_scores and self.use_obj_ptrs_in_encoder:
            self.no_obj_ptr = nn.Parameter(torch.zeros(1, self.hidden_dim))
        self.use_mlp_for_obj_ptr_proj = use_mlp_for_obj_ptr_proj
        self.no_obj_embed_spatial = None
        if no_obj_embed_spatial:
            self.no_obj_embed_spatial = nn.Parameter(torch.zeros(1, self.mem_dim))
        self._build_sam_heads()
        self.max_cond_frames_in_attn = max_cond_frames_in_attn
        self._check_supported()

    def _check_supported(self):
        ok = (self.use_high_res_features_in_sam and self.use_obj_ptrs_in_encoder and self.pred_obj_scores
              and self.fixed_no_obj_ptr and not self.soft_no_obj_ptr and self.proj_tpos_enc_in_obj_ptrs
              and self.add_tpos_enc_to_obj_ptrs and self.directly_add_no_mem_embed
              and not self.multimask_output_in_sam and self.mem_dim < self.hidden_dim and self.num_maskmem > 0)
        if not ok:
            raise NotImplementedError("this build implements the SAM2.1 training configuration "
                                      "(configs/sam2/sam2.1_hiera_t.yaml flags)")

    @property
    def device(self):
        return next(self.parameters()).device

    def _build_sam_heads(self):
        """sam2_base.py:212-260"""
        self.sam_prompt_embed_dim = self.hidden_dim
        self.sam_image_embedding_size = self.image_size // self.backbone_stride
        e = self.sam_image_embedding_size
        self.sam_prompt_encoder = PromptEncoder(embed_dim=self.sam_prompt_embed_dim, image_embedding_size=(e, e),
                                                input_image_size=(self.image_size, self.image_size), mask_in_chans=16)
        self.sam_mask_decoder = MaskDecoder(
            num_multimask_outputs=3,
            transformer=TwoWayTransformer(depth=2, embedding_dim=self.sam_prompt_embed_dim, mlp_dim=2048, num_heads=8),
            transformer_dim=self.sam_prompt_embed_dim, iou_head_depth=3, iou_head_hidden_dim=256,
            use_high_res_features=self.use_high_res_features_in_sam,
            iou_prediction_use_sigmoid=self.iou_prediction_use_sigmoid, pred_obj_scores=self.pred_obj_scores,
            pred_obj_scores_mlp=self.pred_obj_scores_mlp,
            use_multimask_token_for_obj_ptr=self.use_multimask_token_for_obj_ptr,
            **(self.sam_mask_decoder_extra_args or {}))
        if self.use_obj_ptrs_in_encoder:
            self.obj_ptr_proj = (MLP(self.hidden_dim, self.hidden_dim, self.hidden_dim, 3)
                                 if self.use_mlp_for_obj_ptr_proj else Linear(self.hidden_dim, self.hidden_dim))
        else:
            self.obj_ptr_proj = nn.Identity()
        self.obj_ptr_tpos_proj = (Linear(self.hidden_dim, self.mem_dim) if self.proj_tpos_enc_in_obj_ptrs
                                  else nn.Identity())

    # ------------------------------------------------------------ image
    def forward_image(self, img_batch):
        """sam2_base.py:488-506.  img_batch [T, 3, H, W] fp32 (NCHW, as the reference).
        Returns NHWC features: backbone_fpn levels [T, h_i, w_i, C_i] (levels 0/1 projected by
        conv_s0 / conv_s1), vision_pos_enc tables [h_i*w_i, 256]."""
        FN.new_step()  # arena-derived weights (the folded value projections) are rebuilt on first use
        dtype = self.compute_dtype
        x = img_batch.permute(0, 2, 3, 1).contiguous()
        x = ops.cast(x, dtype) if dtype != torch.float32 else x
        enc_requires_grad = any(p.requires_grad for p in self.image_encoder.parameters())
        if enc_requires_grad:
            out = self.image_encoder(x)
        else:
            with torch.no_grad():
                out = self.image_encoder(x)
        fpn = list(out["backbone_fpn"])
        fpn[0] = self.sam_mask_decoder.conv_s0(fpn[0])
        fpn[1] = self.sam_mask_decoder.conv_s1(fpn[1])
        out["backbone_fpn"] = fpn
        return out

    # ------------------------------------------------------- memory bank
    def _obj_pos_table(self, pos_list, max_ptr, dtype, device, repeat=True):
        """temporal encoding of object pointers (sam2_base.py:655-672): sine of the signed frame
        distance / (max_ptr - 1), projected to mem_dim, repeated for the C/mem_dim pointer tokens
        (repeat=False: one row per pointer, the consumer repeats)"""
        key = (tuple(pos_list), max_ptr, dtype, str(device))
        pe = self._tpos_cache.get(key) if hasattr(self, "_tpos_cache") else None
        if pe is None:
            t_diff_max = max_ptr - 1
            pe = get_1d_sine_pe(torch.tensor(pos_list, dtype=torch.float32) / t_diff_max, dim=self.hidden_dim)
            pe = pe.to(device=device, dtype=dtype)
            if not hasattr(self, "_tpos_cache"):
                self._tpos_cache = {}
            self._tpos_cache[key] = pe
        op = self.obj_ptr_tpos_proj(pe)  # [n_ptr, mem_dim]
        return op.repeat_interleave(self.hidden_dim // self.mem_dim, dim=0) if repeat else op

    def _memory_selection(self, frame_idx, num_frames, cond_keys, non_cond_keys, track_in_reverse=False):
        """which bank entries frame `frame_idx` attends to (sam2_base.py:549-647, training order):
        [(t_pos, frame)] spatial memories (conditioning frame first, then t-1, t-2, ...) and
        [(pos, frame)] object pointers -- frame ids only, so the row count of every frame's memory
        is known before the loop runs (the frame-batched backward packs by it)"""
        assert len(cond_keys) > 0 and self.max_cond_frames_in_attn == -1
        mems = [(0, t) for t in cond_keys]
        stride = 1 if self.training else self.memory_temporal_stride_for_eval
        for t_pos in range(1, self.num_maskmem):
            t_rel = self.num_maskmem - t_pos
            if t_rel == 1:
                prev = frame_idx - t_rel if not track_in_reverse else frame_idx + t_rel
            elif not track_in_reverse:
                prev = ((frame_idx - 2) // stride) * stride - (t_rel - 2) * stride
            else:
                prev = -(-(frame_idx + 2) // stride) * stride + (t_rel - 2) * stride
            if prev in non_cond_keys:
                mems.append((t_pos, prev))
        max_ptr = min(num_frames, self.max_obj_ptrs_in_encoder)
        sign = -1 if track_in_reverse else 1
        # eval: only conditioning frames on the tracked side of this frame contribute pointers
        # (only_obj_ptrs_in_the_past_for_eval, sam2_base.py:618-625)
        ptr_cond = [t for t in cond_keys if self.training or not self.only_obj_ptrs_in_the_past_for_eval
                    or (t >= frame_idx if track_in_reverse else t <= frame_idx)]
        ptrs = [((frame_idx - t) * sign if self.use_signed_tpos_enc_to_obj_ptrs else abs(frame_idx - t), t)
                for t in ptr_cond]
        for t_diff in range(1, max_ptr):
            t = frame_idx + t_diff if track_in_reverse else frame_idx - t_diff
            if t < 0 or (num_frames is not None and t >= num_frames):
                break
            if t in non_cond_keys:
                ptrs.append((t_diff, t))
        return mems, ptrs, max_ptr

    def _bank_rows(self, num_frames, L, C):
        """memory rows M_t of frames 1..T-1 (spatial L per memory frame + C/mem_dim tokens per
        object pointer), simulating the bank write / prune of forward_tracking"""
        cond, non_cond, rows = [0], [], []
        for t in range(1, num_frames):
            mems, ptrs, _ = self._memory_selection(t, num_frames, cond, set(non_cond))
            rows.append(len(mems) * L + len(ptrs) * (C // self.mem_dim))
            non_cond.append(t)
            while len(non_cond) > max(self.num_maskmem - 1, 0):
                non_cond.pop(0)
        return rows

    def _prepare_memory_conditioned_features(self, frame_idx, is_init_cond_frame, feat, pos, num_frames,
                                             output_dict, num_objects, track_in_reverse=False, tape=None):
        """sam2_base.py:524-713 (training order).  feat/pos: [L, C] of this frame; returns [O, L, C].
        With a recording `tape` the assembled memory goes into the tape's packed per-frame buffer."""
        L, C = feat.shape
        if is_init_cond_frame:
            x = FN.add_bcast(feat, self.no_mem_embed._s2h_compute.view(-1), bparam=self.no_mem_embed)
            return FN.expand_batch(x.unsqueeze(0), num_objects)
        cond = output_dict["cond_frame_outputs"]
        non_cond = output_dict["non_cond_frame_outputs"]
        mems, ptr_sel, max_ptr = self._memory_selection(frame_idx, num_frames, list(cond), set(non_cond),
                                                        track_in_reverse)
        bank = lambda t: cond[t] if t in cond else non_cond[t]  # noqa: E731
        feats = [bank(t)["maskmem_features"].reshape(num_objects, -1, self.mem_dim) for _, t in mems]
        spatial_pos = bank(mems[-1][1])["maskmem_pos_enc"]
        tpos_idx = [self.num_maskmem - t_pos - 1 for t_pos, _ in mems]
        pos_list = [p for p, _ in ptr_sel]
        ptrs = [bank(t)["obj_ptr"] for _, t in ptr_sel]
        n_ptr_tok = len(ptrs) * (C // self.mem_dim)
        if not ptrs:  # eval, tracking away from every conditioning frame (sam2_base.py:677)
            raise NotImplementedError("memory attention without object-pointer tokens")
        if tape is not None:
            if self.obj_ptr_tpos_proj.weight.requires_grad:
                raise NotImplementedError("frame-batched backward with a trainable obj_ptr_tpos_proj")
            with torch.no_grad():  # one row per pointer: the tape's memory_pos writes each into its k rows
                obj_pos = self._obj_pos_table(pos_list, max_ptr, feat.dtype, feat.device, repeat=False)
            obj_rep = C // self.mem_dim
            M = sum(f.shape[1] for f in feats) + n_ptr_tok
            memory = tape.varlen_slot("memory", (num_objects, M, self.mem_dim), feat.dtype)
            r, pairs = 0, []
            for f in feats:
                pairs.append((f, memory[:, r:r + f.shape[1]]))
                r += f.shape[1]
            k = C // self.mem_dim  # each pointer [O, C] fills k memory rows of mem_dim (the stack + reshape)
            for i, ptr in enumerate(ptrs):
                pairs.append((ptr, memory[:, r + k * i:r + k * (i + 1)].view(num_objects, C)))
            ops.copy_segments(pairs)  # one launch for the whole bank
        else:
            obj_pos = self._obj_pos_table(pos_list, max_ptr, feat.dtype, feat.device)
            obj_rep = 1
            ptr_tokens = torch.stack(ptrs, dim=1).reshape(num_objects, n_ptr_tok, self.mem_dim)
            memory = torch.cat(feats + [ptr_tokens], dim=1)
        mpos = FN_memory_pos(self.maskmem_tpos_enc, obj_pos, spatial_pos, tpos_idx, spatial_pos.shape[0], feat.dtype,
                             obj_rep)
        return self.memory_attention(feat, pos, memory, mpos, num_obj_ptr_tokens=n_ptr_tok, num_objects=num_objects)

    # ------------------------------------------------------------ heads
    def _forward_sam_heads(self, pix, prompt, high_res, num_objects, dense=None):
        """sam2_base.py:262-434 (single mask).  pix [O, L, C]; prompt (pe [O, N, C] f32, labels [O, N]
        int32) on the device; high_res (s0, s1) NHWC (batch 1 = broadcast over objects); `dense` an
        optional mask-prompt embedding [O, L, C] (prompt_encoder._embed_masks, the predictor's
        refinement clicks) in place of no_mask_embed."""
        O = num_objects
        h = w = self.sam_image_embedding_size
        dt = pix.dtype
        pe_dev, lab_dev = prompt
        sparse = self.sam_prompt_encoder.sparse(pe_dev, lab_dev, dt)
        dense_pe = self.sam_prompt_encoder.dense_pe_table(pix.device, dt)
        defer = pix.dtype == torch.bfloat16 and hasattr(self.obj_ptr_proj, "layers")
        masks, ious, token0, score = self.sam_mask_decoder(pix, h, w, dense_pe, sparse,
                                                           self.sam_prompt_encoder.no_mask_embed, high_res,
                                                           **({"dense": dense} if dense is not None else {}),
                                                           defer_score=defer)
        ptr = None
        if defer:  # object-score head and object-pointer projection: no gradient, one launch for both
            with torch.no_grad():
                score, ptr = FN.mlp_heads_nograd([(self.sam_mask_decoder.pred_obj_score_head, score),
                                                  (self.obj_ptr_proj, token0.detach())])
                score = ops.cast(score, torch.float32)
        score_flat = score.view(-1).contiguous()
        low = FN.cast_gate(masks, torch.float32, score_flat, NO_OBJ_SCORE)
        low = low.view(O, 4 * h, 4 * w)
        high = FN.bilinear(low, self.image_size, self.image_size)
        with torch.no_grad():
            if ptr is None:
                ptr = self.obj_ptr_proj(token0.detach())
            ptr = ops.gate_mix(ptr, score_flat, self.no_obj_ptr._s2h_compute.view(-1), scale_x=self.fixed_no_obj_ptr)
        return low, high, ious, ptr, score

    @torch.no_grad()
    def _use_mask_as_output(self, feat, masks, score, high_res, num_objects):
        """sam2_base.py:436-486 (mask prompt on the conditioning frame): the object masks as output
        logits (x20 - 10), antialiased bilinear /4 for the low-res, IoU prediction 1, and an object
        pointer from the SAM heads run on the RAW backbone feature (no no_mem_embed) with
        mask_downsample(mask) as the mask prompt; pointer gated by mask non-emptiness.  masks
        [O, H, W] f32 on the device; score [O] = 20 * any(mask) - 10 (host-computed).  No
        gradient reaches anything here (constant outputs, detached pointer)."""
        from ...kernels.functional_sam import aa_downsample
        O = num_objects
        h = w = self.sam_image_embedding_size
        H = self.image_size
        dt = self.compute_dtype
        high = ops.act_fwd(masks.reshape(O, H * H), None, scale=20.0, shift=-10.0)
        low = aa_downsample(high.view(O, H, H), H // 4, H // 4).view(O, -1)
        ious = torch.ones(O, 1, device=masks.device)
        # mask_downsample: Conv2d(1, 1, 4, 4) as an im2col GEMM on the [O, H, W, 1] mask
        m = ops.cast(masks.reshape(O, H, H, 1), dt) if dt != torch.float32 else masks.reshape(O, H, H, 1)
        col, Ho, Wo = ops.im2col(m.contiguous(), 4, 4, 4, 0)
        md = ops.linear(col, self.mask_downsample.compute_weight(), self.mask_downsample.compute_bias())
        dense = self.sam_prompt_encoder.dense_from_mask(md.view(O, Ho, Wo, 1), dt)
        pix = FN.expand_batch(feat.unsqueeze(0), O)
        pe1, lab1 = self._mask_pad_prompt
        sparse = self.sam_prompt_encoder.sparse(pe1, lab1, dt)
        dense_pe = self.sam_prompt_encoder.dense_pe_table(pix.device, dt)
        _, _, token0, _ = self.sam_mask_decoder(pix, h, w, dense_pe, sparse, self.sam_prompt_encoder.no_mask_embed,
                                                high_res, dense=dense)
        ptr = self.obj_ptr_proj(token0)
        ptr = ops.gate_mix(ptr, score, self.no_obj_ptr._s2h_compute.view(-1), scale_x=self.fixed_no_obj_ptr)
        return low, high, ious, ptr, score.view(O, 1)

    def _encode_new_memory(self, feat, high_res, score, num_objects):
        """sam2_base.py:715-769 (training): sigmoid(logits)*scale+bias -> memory encoder ->
        + no-object spatial embedding where the object is predicted absent."""
        h = w = self.sam_image_embedding_size
        with torch.no_grad():
            m = high_res.detach().view(num_objects, self.image_size, self.image_size)
            mfeat, mpos = self.memory_encoder(feat, m, h, w, scale=self.sigmoid_scale_for_mem_enc,
                                              shift=self.sigmoid_bias_for_mem_enc)
            if self.no_obj_embed_spatial is not None:
                mfeat = ops.gate_mix(mfeat.view(num_objects, -1), score.view(-1).contiguous(),
                                     self.no_obj_embed_spatial._s2h_compute.view(-1)).view(mfeat.shape)
        return mfeat, mpos


def FN_memory_pos(tpos_param, obj_pos, spatial_pos, tpos_idx, L, dtype, obj_rep=1):
    from ...kernels.functional_sam import memory_pos
    return memory_pos(tpos_param, obj_pos, spatial_pos, tpos_idx, L, dtype, obj_rep)


_ = math
