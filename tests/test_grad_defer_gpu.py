"""Deferred fixed-order gradient sums (csrc/grad_defer.hip, ops.deferred_grad_sums): inside the scope the
second pass of LayerNorm gamma / beta and column-sum bias gradients whose destination is in the sink is
recorded and run at the scope's end; destinations outside the sink keep the immediate pass."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _ops():
    from sam2_video.kernels import ops
    ops.wgrad_workspace(torch.device(DEV))  # the immediate fixed-order path's workspace
    return ops


def _close(a, b, tol=2e-6):
    err = (a - b).abs().max().item()
    assert err <= tol * (b.abs().max().item() + 1e-12), err


def test_deferred_sums_match_immediate():
    ops = _ops()
    from sam2_video.kernels._lib import lib
    torch.manual_seed(0)
    C = 256
    x = torch.randn(13312, C, device=DEV).to(torch.bfloat16)
    dy = torch.randn(13312, C, device=DEV).to(torch.bfloat16)
    gamma = torch.randn(C, device=DEV)
    mean = x.float().mean(-1).contiguous()
    rstd = (x.float().var(-1, unbiased=False) + 1e-5).rsqrt().contiguous()
    g = torch.randn(93184, 768, device=DEV).to(torch.bfloat16)
    outs = {}
    for mode in ("immediate", "deferred"):
        torch.manual_seed(1)  # the same starting gradients in both modes
        arena = torch.randn(4096, device=DEV)  # the sink: gamma / beta / bias gradient slots inside
        outside = torch.randn(768, device=DEV)  # not in the sink: immediate in both modes
        a0 = arena.clone()
        dg, db, gb = arena[:C], arena[C:2 * C], arena[1024:1024 + 768]
        if mode == "deferred":
            with ops.deferred_grad_sums(arena):
                ops.layernorm_bwd(x, dy, gamma, mean, rstd, dgamma=dg, dbeta=db)
                ops.colsum(g, gb)
                ops.colsum(g[:5000], gb)  # a second sum into the same slots: a later launch, in order
                ops.colsum(g, outside)
                assert lib().s2h_grad_defer_pending() == 3
                torch.cuda.synchronize()
                _close(outside, outs["immediate"][2])  # outside the sink: already summed
                assert torch.equal(arena[:2 * C], a0[:2 * C])  # deferred: not yet touched
            assert lib().s2h_grad_defer_pending() == 0
        else:
            ops.layernorm_bwd(x, dy, gamma, mean, rstd, dgamma=dg, dbeta=db)
            ops.colsum(g, gb)
            ops.colsum(g[:5000], gb)
            ops.colsum(g, outside)
        torch.cuda.synchronize()
        outs[mode] = (arena.clone(), a0, outside.clone())
    (ai, a0i, _), (ad, a0d, _) = outs["immediate"], outs["deferred"]
    _close(ad - a0d, ai - a0i, 1e-5)
    assert torch.equal(ad[2 * C:1024], a0d[2 * C:1024])  # untouched slots


def test_deferred_sums_repeat_bitwise_and_small_workspace():
    """the same records give bit-identical sums; a workspace too small for all of them flushes early
    (in record order) and still gives the same result"""
    ops = _ops()
    from sam2_video.kernels._lib import call, lib
    torch.manual_seed(1)
    gs = [torch.randn(20000 + 1000 * i, 512, device=DEV).to(torch.bfloat16) for i in range(6)]
    res = []
    for ws_bytes in (64 << 20, 64 << 20, 1 << 20):
        arena = torch.zeros(2048, device=DEV)
        ws = torch.empty(ws_bytes // 4, device=DEV)
        call("s2h_grad_defer", ws.data_ptr(), ws_bytes, arena.data_ptr(), arena.numel() * 4)
        try:
            for i, g in enumerate(gs):
                ops.colsum(g, arena[512 * (i % 3):512 * (i % 3) + 512])
            if ws_bytes == 1 << 20:
                assert lib().s2h_grad_defer_pending() < len(gs)  # early flushes happened
        finally:
            call("s2h_grad_defer_flush", ops.stream())
            call("s2h_grad_defer", None, 0, None, 0)
        torch.cuda.synchronize()
        res.append(arena.clone())
    assert torch.equal(res[0], res[1])
    ref = torch.zeros(2048, device=DEV, dtype=torch.float64)
    for i, g in enumerate(gs):
        ref[512 * (i % 3):512 * (i % 3) + 512] += g.double().sum(0)
    _close(res[0].double(), ref, 1e-5)
    _close(res[2].double(), ref, 1e-5)


def test_scope_close_with_pending_records_is_refused():
    _ops()
    from sam2_video.kernels._lib import lib
    torch.manual_seed(2)
    arena = torch.zeros(256, device=DEV)
    ws = torch.empty(1 << 18, device=DEV)
    h = lib()
    assert h.s2h_grad_defer(ws.data_ptr(), ws.numel() * 4, arena.data_ptr(), 1024) == 0
    from sam2_video.kernels import ops
    ops.colsum(torch.randn(4096, 256, device=DEV).to(torch.bfloat16), arena)
    assert h.s2h_grad_defer_pending() == 1
    assert h.s2h_grad_defer(None, 0, None, 0) != 0  # records pending: refused
    assert h.s2h_grad_defer_flush(ops.stream()) == 0
    assert h.s2h_grad_defer(None, 0, None, 0) == 0


def test_records_from_a_second_stream_keep_the_immediate_pass_and_reset_ends_a_failed_scope():
    """one stream per scope -- a column sum issued on another stream (the opt-in weight-gradient
    side stream) is not deferred (its immediate second pass runs on its own stream); a flush on a stream
    other than the records' is refused, and s2h_grad_defer_reset ends the scope so the next can register"""
    ops = _ops()
    from sam2_video.kernels._lib import lib
    torch.manual_seed(3)
    h = lib()
    arena = torch.zeros(512, device=DEV)
    ws = torch.empty(1 << 18, device=DEV)
    g = torch.randn(4096, 256, device=DEV).to(torch.bfloat16)
    side = torch.cuda.Stream()
    assert h.s2h_grad_defer(ws.data_ptr(), ws.numel() * 4, arena.data_ptr(), arena.numel() * 4) == 0
    try:
        ops.colsum(g, arena[:256])  # main stream: deferred
        assert h.s2h_grad_defer_pending() == 1
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            ops.colsum(g, arena[256:])  # other stream: immediate
        assert h.s2h_grad_defer_pending() == 1
        torch.cuda.current_stream().wait_stream(side)
        assert h.s2h_grad_defer_flush(side.cuda_stream) != 0  # not the records' stream: refused
        assert h.s2h_grad_defer_pending() == 1
        assert h.s2h_grad_defer_flush(ops.stream()) == 0
    finally:
        h.s2h_grad_defer_reset()
    torch.cuda.synchronize()
    ref = g.double().sum(0)
    _close(arena[:256].double(), ref, 1e-5)
    _close(arena[256:].double(), ref, 1e-5)
    # a failed flush inside ops.deferred_grad_sums still ends the scope (reset in its finally)
    assert h.s2h_grad_defer(ws.data_ptr(), ws.numel() * 4, arena.data_ptr(), arena.numel() * 4) == 0
    ops.colsum(g, arena[:256])
    h.s2h_grad_defer_reset()  # drops the pending record
    assert h.s2h_grad_defer_pending() == 0
    with ops.deferred_grad_sums(arena):
        ops.colsum(g, arena[:256])
    assert h.s2h_grad_defer_pending() == 0


def test_persistent_buffers_refuse_first_use_inside_a_capture():
    """the library keeps the addresses of the weight-gradient workspace and the deferral
    workspace for the whole process; first allocated inside a graph capture they would come from the
    graph's private pool and dangle once the graph is released -- refused loudly instead"""
    ops = _ops()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g):
            with pytest.raises(RuntimeError, match="inside a HIP graph capture"):
                ops._persistent_alloc("wgrad_workspace", 16, torch.float32, "cuda")
