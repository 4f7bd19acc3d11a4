"""Lightning 2.x automatic optimization, restated for the tests (Lightning is not installed in this
image): the order in which `lightning.pytorch`'s fit loop calls a LightningModule's hooks.

Per micro-batch (`_AutomaticOptimization.run` / `Closure.closure`):
  1. closure: out = training_step(batch, batch_idx); closure_loss = out / accumulate_grad_batches
     (ClosureResult.from_training_step_output); on the first batch of a window
     (batch_idx % accumulate == 0) optimizer.zero_grad() -- AFTER training_step, BEFORE backward;
     then the precision plugin scales the loss (GradScaler.scale for "16-mixed") and calls
     module.backward(scaled_loss);
  2. if fit_loop._should_accumulate() (not the window's last batch, not the epoch's last): only the
     closure runs;
  3. else the optimizer step: with a GradScaler (MixedPrecision.optimizer_step) closure(), then
     scaler.unscale_(optimizer) unless the optimizer handles unscaling, then the clip hook
     (configure_gradient_clipping), scaler.step(optimizer) (skips the step on inf / NaN) and
     scaler.update(); without one optimizer.step(closure) whose closure runs the clip hook after
     the backward (Precision._wrap_closure); then the per-step LR scheduler.
"""
from types import SimpleNamespace


class StubFitLoop:
    def __init__(self, acc, n_batches):
        self.acc, self.n = acc, n_batches
        self.batch_idx = 0

    def _should_accumulate(self):
        last = self.batch_idx + 1 >= self.n
        return (self.batch_idx + 1) % self.acc != 0 and not last


def make_trainer(acc, n_batches, clip, precision="32-true", scaler=None, stepping_batches=None):
    tr = SimpleNamespace(accumulate_grad_batches=acc, gradient_clip_val=clip, precision=precision,
                         estimated_stepping_batches=stepping_batches or -(-n_batches // acc),
                         num_training_batches=n_batches)
    tr.fit_loop = StubFitLoop(acc, n_batches)
    tr.precision_plugin = SimpleNamespace(scaler=scaler)
    return tr


def lightning_fit(mod, tr, batches, on_step=None):
    """drive `mod` (with `mod._trainer = tr`) over `batches` as Lightning's automatic optimization
    does; returns the optimizer.  on_step(i) is called after each optimizer step."""
    conf = mod.configure_optimizers()
    opt, sched = conf["optimizer"], conf["lr_scheduler"]["scheduler"] if "lr_scheduler" in conf else None
    acc, clip = tr.accumulate_grad_batches, tr.gradient_clip_val
    scaler = tr.precision_plugin.scaler
    n = len(batches)
    for i, batch in enumerate(batches):
        tr.fit_loop.batch_idx = i

        def closure(i=i, batch=batch):
            out = mod.training_step(batch, i)
            closure_loss = out / acc
            if i % acc == 0:
                opt.zero_grad()
            mod.backward(scaler.scale(closure_loss) if scaler is not None else closure_loss)
            return closure_loss

        if tr.fit_loop._should_accumulate():
            closure()
            continue
        if scaler is not None:
            closure()
            if not getattr(opt, "_step_supports_amp_scaling", False):
                scaler.unscale_(opt)
            mod.configure_gradient_clipping(opt, clip, "norm")
            scaler.step(opt)
            scaler.update()
        else:
            def wrapped():
                out = closure()
                mod.configure_gradient_clipping(opt, clip, "norm")
                return out
            opt.step(closure=wrapped)
        if sched is not None:
            sched.step()
        if on_step is not None:
            on_step(i)
    assert n == len(batches)
    return opt
