"""Shared test helpers (not a test module)."""
from __future__ import annotations

import contextlib

import numpy as np


@contextlib.contextmanager
def engine_options(**opts):
    """Process-wide engine options (fqlpop_set_engine_option) for the Population
    handles created inside the block; restored to the defaults afterwards."""
    from fqlpop import reset_engine_options, set_engine_option
    try:
        for k, v in opts.items():
            set_engine_option(k, v)
        yield
    finally:
        reset_engine_options()


# Adam moments may differ from the float64 oracle's by this fraction of each leaf's scale
# (max |oracle value|): the GPU accumulates in fp32, and the critic's first-layer
# gradient passes through four LayerNorm backwards (measured up to 1.7e-4 at B = 1024;
# the bound is 1.5x that).
MOMENT_REL = 2.5e-4


class OptimiserChecker:
    """Per-step parity of one member's update, split in two exact parts:

    1. gradients: the Adam moments m_t and v_t of every leaf against the oracle's, within
       MOMENT_REL of the leaf's scale (this covers every gradient element, small leaves too);
    2. the optimiser itself: the GPU's new parameters against optax.adam (eps outside the
       sqrt, bias corrections with count t) applied in float64 to the GPU's OWN previous
       parameters and new moments, and target_critic against the EMA of the GPU's own
       pre-update critic and target -- tight (1e-7 + 1e-6 |p|), so a skipped, partial or
       wrong update of any leaf fails, independently of how well-conditioned its
       gradient is.

    Adam normalises each update, so comparing parameters with the oracle's directly is
    ill-conditioned where a gradient element is ~0; that comparison is kept only as a
    bound (2 lr per step).  Call ``before()`` ahead of each step and ``after(...)`` after.
    """

    def __init__(self, pop, member, lr, tau, b1=0.9, b2=0.999, eps=1e-8):
        self.pop, self.member, self.lr, self.tau = pop, member, lr, tau
        self.b1, self.b2, self.eps = b1, b2, eps
        self.prev = None

    def _state(self):
        from fqlpop._lib import STATE_ADAM_M, STATE_ADAM_V, STATE_PARAMS
        return tuple(self.pop.get_flat(self.member, w).astype(np.float64)
                     for w in (STATE_PARAMS, STATE_ADAM_M, STATE_ADAM_V))

    def before(self):
        self.prev = self._state()
        self.count0 = self.pop.get_count(self.member)

    def after(self, params_o, opt_o, steps_done, tag):
        p0, _, _ = self.prev
        p1, m1, v1 = self._state()
        t = self.pop.get_count(self.member)
        assert t == self.count0 + 1, f"{tag}: count {self.count0} -> {t}"
        bc1, bc2 = 1.0 - self.b1 ** t, 1.0 - self.b2 ** t
        bad = []
        for name, off, shape in self.pop.leaves:
            net, leaf = name.split("/", 1)
            sl = slice(off, off + int(np.prod(shape)))
            for what, got, want in (("m", m1, opt_o["m"]), ("v", v1, opt_o["v"])):
                o = np.asarray(want[net][leaf], dtype=np.float64).reshape(-1)
                scale = float(np.abs(o).max()) if o.size else 0.0
                err = float(np.abs(got[sl] - o).max()) if o.size else 0.0
                if err > MOMENT_REL * scale + 1e-30:
                    bad.append(f"{name} adam {what}: max err {err:.3g} vs leaf scale {scale:.3g}")
            if net == "target_critic":
                coff = next(o for n, o, _ in self.pop.leaves if n == "critic/" + leaf)
                want_p = self.tau * p0[coff:coff + (sl.stop - sl.start)] + (1.0 - self.tau) * p0[sl]
            else:
                want_p = p0[sl] - self.lr * (m1[sl] / bc1) / (np.sqrt(v1[sl] / bc2) + self.eps)
            d = np.abs(p1[sl] - want_p)
            if d.size and np.any(d > 1e-7 + 1e-6 * np.abs(want_p)):
                bad.append(f"{name} optimiser: max |p - adam(own p, m, v)| {float(d.max()):.3g}")
            o = np.asarray(params_o[net][leaf], dtype=np.float64).reshape(-1)
            d = np.abs(p1[sl] - o)
            if d.size and float(d.max()) > 2 * self.lr * steps_done + 1e-5:
                bad.append(f"{name} params: max diff from oracle {float(d.max()):.3g} > 2 lr per step")
        assert not bad, f"{tag}:\n" + "\n".join(bad[:20])
