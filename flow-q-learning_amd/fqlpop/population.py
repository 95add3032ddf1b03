"""Population engine: one libfqlpop handle = an alpha-population of FQL agents on one GPU.

Every call below advances ALL active members with one set of member-batched
HIP launches.  This is the object the reference-shaped
surface (``fql.agents.fql.FQLAgent``, ``trainer.Trainer``) drives; it mirrors
the reference call sites it replaces:

* ``Population.step``            <- ``Experiment.train`` loop body
                                    (reference trainer/experiment.py:106-109)
* ``Population.total_loss``      <- ``agent.total_loss(val_batch, grad_params=None)``
                                    (trainer/experiment.py:114-115)
* ``Population.sample_actions``  <- ``agent.sample_actions`` (evaluator/evaluation.py:58-64)
* ``Population.state_dict``      <- ``flax.serialization.to_state_dict(agent)``
                                    (trainer/experiment.py:92,135)
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from fqlpop import _lib
from fqlpop._lib import (INFO_STRIDE, STATE_ADAM_M, STATE_ADAM_V, STATE_PARAMS,
                         TRAIN_INFO_KEYS, VAL_INFO_KEYS, check, fptr)


@dataclass
class PopulationConfig:
    """The AgentConfig fields (reference trainer/config.py:5-22) the update reads."""
    obs_dim: int = 28
    action_dim: int = 5
    hidden_dims: tuple = (512, 512, 512, 512)
    batch_size: int = 256
    num_qs: int = 2
    layer_norm: bool = True
    actor_layer_norm: bool = False
    flow_steps: int = 10
    q_agg: str = "mean"
    normalize_q_loss: bool = False
    discount: float = 0.99
    tau: float = 0.005
    lr: float = 3e-4
    use_graph: bool = True

    def to_c(self) -> _lib.Config:
        hd = tuple(self.hidden_dims)
        if len(set(hd)) != 1:
            raise ValueError(f"hidden_dims must be uniform, got {hd}")
        if self.q_agg not in ("mean", "min"):
            raise ValueError(f"q_agg must be 'mean' or 'min', got {self.q_agg!r}")
        return _lib.Config(
            obs_dim=int(self.obs_dim), action_dim=int(self.action_dim),
            hidden_dim=int(hd[0]), num_hidden=len(hd), batch_size=int(self.batch_size),
            num_qs=int(self.num_qs), layer_norm=int(bool(self.layer_norm)),
            actor_layer_norm=int(bool(self.actor_layer_norm)), flow_steps=int(self.flow_steps),
            q_agg_min=int(self.q_agg == "min"), normalize_q_loss=int(bool(self.normalize_q_loss)),
            discount=float(self.discount), tau=float(self.tau), lr=float(self.lr),
            use_graph=int(bool(self.use_graph)))

    @classmethod
    def from_agent_config(cls, cfg: dict, obs_dim: int, action_dim: int, **kw):
        """From an ``asdict(AgentConfig)`` dict (reference trainer/config.py:5-22)."""
        if tuple(cfg.get("actor_hidden_dims", (512,) * 4)) != tuple(cfg.get("value_hidden_dims", (512,) * 4)):
            raise ValueError("actor_hidden_dims must equal value_hidden_dims")
        if cfg.get("encoder") not in (None, "None"):
            raise ValueError("visual encoders are out of scope (encoder must be None)")
        return cls(obs_dim=obs_dim, action_dim=action_dim,
                   hidden_dims=tuple(cfg.get("value_hidden_dims", (512,) * 4)),
                   batch_size=int(cfg.get("batch_size", 256)),
                   layer_norm=bool(cfg.get("layer_norm", True)),
                   actor_layer_norm=bool(cfg.get("actor_layer_norm", False)),
                   flow_steps=int(cfg.get("flow_steps", 10)), q_agg=cfg.get("q_agg", "mean"),
                   normalize_q_loss=bool(cfg.get("normalize_q_loss", False)),
                   discount=float(cfg.get("discount", 0.99)), tau=float(cfg.get("tau", 0.005)),
                   lr=float(cfg.get("lr", 3e-4)), **kw)


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


SPLIT_SITES = ("bc_forward", "euler_flow", "onestep_forward", "target_critic", "critic_forward", "critic_backward",
               "onestep_backward", "critic_backward_td")


def split_plan(cfg: "PopulationConfig", n_members: int) -> dict:
    """The split plan (fqlpop_split_plan; no GPU call) of an n_members population with
    ``cfg`` under the current engine options: blocks per 16-column tile per launch site
    (1 = unsplit) and whether the small-population schedule runs."""
    c = cfg.to_c()
    F = (ctypes.c_int * 8)()
    small = ctypes.c_int()
    check(_lib.load_library().fqlpop_split_plan(ctypes.byref(c), int(n_members), F, ctypes.byref(small)))
    out = dict(zip(SPLIT_SITES, [int(x) for x in F]))
    out["small_sched"] = bool(small.value)
    return out


class Population:
    """A population of FQL agents (one alpha and seed per member) on one GPU."""

    def __init__(self, cfg: PopulationConfig, alphas, seeds, device: int = 0):
        self.lib = _lib.load_library()
        self.cfg = cfg
        alphas = _f32(alphas).reshape(-1)
        seeds = np.ascontiguousarray(np.asarray(seeds, dtype=np.uint64).reshape(-1))
        if alphas.shape != seeds.shape:
            raise ValueError("alphas and seeds must have the same length")
        self.n = int(alphas.shape[0])
        self.alphas = alphas.copy()
        self.seeds = seeds.copy()
        self._c = cfg.to_c()
        # the engine reads its options at create: hand it this process's GPU_MAX_HW_QUEUES for
        # this create only (the option is process-wide; later populations see the old value)
        hwq = _lib.hw_queues_from_env()
        prev_hwq = _lib.get_engine_option("hw_queues") if hwq is not None else None
        if hwq is not None:
            _lib.set_engine_option("hw_queues", hwq)
        h = ctypes.c_void_p()
        try:
            check(self.lib.fqlpop_create(ctypes.byref(self._c), self.n, fptr(alphas),
                                         seeds.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                         int(device), ctypes.byref(h)))
        finally:
            if prev_hwq is not None:
                _lib.set_engine_option("hw_queues", prev_hwq)
        self._h = h
        self.active = np.ones(self.n, dtype=bool)
        n = ctypes.c_int64()
        check(self.lib.fqlpop_state_size(self._h, ctypes.byref(n)))
        self.state_size = int(n.value)
        self.leaves = self._leaf_table()

    # ------------------------------------------------------------------ misc
    def close(self):
        if getattr(self, "_h", None):
            check(self.lib.fqlpop_destroy(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def flops_per_member_step(self) -> float:
        return float(self.lib.fqlpop_flops_per_member_step(ctypes.byref(self._c)))

    def sync(self):
        check(self.lib.fqlpop_sync(self._h))

    def _leaf_table(self):
        n = ctypes.c_int()
        check(self.lib.fqlpop_num_leaves(self._h, ctypes.byref(n)))
        out = []
        name = ctypes.create_string_buffer(256)
        off = ctypes.c_int64()
        nd = ctypes.c_int()
        shp = (ctypes.c_int64 * 3)()
        for i in range(n.value):
            check(self.lib.fqlpop_leaf_info(self._h, i, name, 256, ctypes.byref(off),
                                            ctypes.byref(nd), shp))
            out.append((name.value.decode(), int(off.value), tuple(int(shp[k]) for k in range(nd.value))))
        return out

    # --------------------------------------------------------------- dataset
    def set_dataset(self, data: dict, which: str = "train"):
        """``data``: dict with observations, actions, rewards, masks,
        next_observations (row-major, any float dtype; torch CUDA tensors on
        this device are used in place)."""
        keys = ("observations", "actions", "rewards", "masks", "next_observations")
        on_dev = all(hasattr(data[k], "is_cuda") and data[k].is_cuda for k in keys)
        if on_dev:
            arrs = [data[k].contiguous().float() for k in keys]
            ptrs = [ctypes.c_void_p(a.data_ptr()) for a in arrs]
            n = int(arrs[0].shape[0])
        else:
            arrs = [_f32(data[k]) for k in keys]
            ptrs = [a.ctypes.data_as(ctypes.c_void_p) for a in arrs]
            n = int(arrs[0].shape[0])
        check(self.lib.fqlpop_set_dataset(self._h, 0 if which == "train" else 1, *ptrs, n, int(on_dev)))

    # ---------------------------------------------------------------- active
    def set_active(self, mask):
        m = np.ascontiguousarray(np.asarray(mask, dtype=np.uint8).reshape(-1))
        if m.shape[0] != self.n:
            raise ValueError("mask length must equal the population size")
        check(self.lib.fqlpop_set_active(self._h, m.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))))
        self.active = m.astype(bool)

    @property
    def active_ids(self):
        return [int(i) for i in np.nonzero(self.active)[0]]

    # ------------------------------------------------------------ hot path
    def step(self, n_steps: int = 1):
        """n_steps population updates (device-side sampling) of every active member."""
        check(self.lib.fqlpop_step(self._h, int(n_steps)))

    def _pack_batches(self, batches):
        B = self.cfg.batch_size
        D, A = self.cfg.obs_dim, self.cfg.action_dim
        parts = []
        for b in batches:
            parts += [_f32(b["observations"]).reshape(B * D), _f32(b["actions"]).reshape(B * A),
                      _f32(b["rewards"]).reshape(B), _f32(b["masks"]).reshape(B),
                      _f32(b["next_observations"]).reshape(B * D)]
        return np.concatenate(parts)

    def _pack_noises(self, noises):
        if noises is None:
            return None
        B, A = self.cfg.batch_size, self.cfg.action_dim
        parts = []
        for nz in noises:
            parts += [_f32(nz["z_next"]).reshape(B * A), _f32(nz["x0"]).reshape(B * A),
                      _f32(nz["t"]).reshape(B), _f32(nz["z_d"]).reshape(B * A),
                      _f32(nz["z_metric"]).reshape(B * A)]
        return np.concatenate(parts)

    def _check_count(self, items, what):
        if items is not None and len(items) != len(self.active_ids):
            raise ValueError(f"one {what} per active member ({len(self.active_ids)}), got {len(items)}")

    def step_injected(self, batches, noises=None):
        """One update of every active member (in slot order) on the given host
        batches.  ``noises`` None: drawn on device; else the parity mode (see
        oracle/fql_oracle.py for the keys)."""
        self._check_count(batches, "batch")
        self._check_count(noises, "noise dict")
        pb = self._pack_batches(batches)
        pn = self._pack_noises(noises)
        check(self.lib.fqlpop_step_injected(self._h, fptr(pb), None if pn is None else fptr(pn)))

    def total_loss(self, batches=None, noises=None):
        """Validation losses of every active member; returns {member: info}.
        ``batches`` None: sampled on device from the val dataset."""
        if batches is None:
            if noises is not None:
                raise ValueError("noises need batches")
            check(self.lib.fqlpop_total_loss(self._h, None, None))
        else:
            self._check_count(batches, "batch")
            self._check_count(noises, "noise dict")
            pb = self._pack_batches(batches)
            pn = self._pack_noises(noises)
            check(self.lib.fqlpop_total_loss(self._h, fptr(pb), None if pn is None else fptr(pn)))
        return self.read_info("val")

    def read_info_array(self, which: str = "train") -> np.ndarray:
        out = np.zeros((self.n, INFO_STRIDE), dtype=np.float32)
        check(self.lib.fqlpop_read_info(self._h, 0 if which == "train" else 1, fptr(out)))
        return out

    def read_info(self, which: str = "train") -> dict:
        arr = self.read_info_array(which)
        keys = TRAIN_INFO_KEYS if which == "train" else VAL_INFO_KEYS
        return {i: {k: float(arr[i, j]) for j, k in enumerate(keys)} for i in self.active_ids}

    def sample_actions(self, member: int, observations, noise=None, seed: int = 0) -> np.ndarray:
        obs = _f32(observations)
        squeeze = obs.ndim == 1
        obs = obs.reshape(-1, self.cfg.obs_dim)
        n = obs.shape[0]
        out = np.zeros((n, self.cfg.action_dim), dtype=np.float32)
        nz = None if noise is None else _f32(noise).reshape(n, self.cfg.action_dim)
        check(self.lib.fqlpop_sample_actions(self._h, int(member), fptr(obs), n,
                                             None if nz is None else fptr(nz),
                                             ctypes.c_uint64(int(seed) & (2**64 - 1)), fptr(out)))
        return out[0] if squeeze else out

    # ------------------------------------------------------ world-model eval
    def set_env_model(self, sp_flat, tp_flat, sp_hidden=(128, 256, 128), tp_hidden=(128, 128)):
        """Upload a BaselineStatePredictor / TerminationPredictor pair as flat
        flax-ordered parameter vectors (envmodel.flatten_state_predictor / ...)."""
        c = _lib.EnvModelConfig()
        c.obs_dim, c.action_dim = self.cfg.obs_dim, self.cfg.action_dim
        c.sp_num_hidden = len(sp_hidden)
        c.tp_num_hidden = len(tp_hidden)
        for i, d in enumerate(sp_hidden):
            c.sp_hidden[i] = int(d)
        for i, d in enumerate(tp_hidden):
            c.tp_hidden[i] = int(d)
        n_sp, n_tp = ctypes.c_int64(), ctypes.c_int64()
        check(self.lib.fqlpop_envmodel_param_count(ctypes.byref(c), ctypes.byref(n_sp), ctypes.byref(n_tp)))
        sp = _f32(sp_flat).reshape(-1)
        tp = _f32(tp_flat).reshape(-1)
        if sp.shape[0] != n_sp.value or tp.shape[0] != n_tp.value:
            raise ValueError(f"env-model sizes {sp.shape[0]}/{tp.shape[0]} != expected {n_sp.value}/{n_tp.value}")
        check(self.lib.fqlpop_set_env_model(self._h, ctypes.byref(c), fptr(sp), sp.shape[0], fptr(tp), tp.shape[0]))
        self._em_cfg = c

    def rollout(self, init_obs, max_steps: int, seed: int = 0, noise=None, return_obs: bool = False):
        """World-model evaluation of every ACTIVE member in one launch.

        Returns (success [n_active, n_envs], lengths [n_active, n_envs]) and,
        with return_obs, the observations after the last step [n_active, n_envs, obs]."""
        obs = _f32(init_obs).reshape(-1, self.cfg.obs_dim)
        n_envs = obs.shape[0]
        na = len(self.active_ids)
        nz = None
        if noise is not None:
            nz = _f32(noise).reshape(na, int(max_steps), n_envs, self.cfg.action_dim)
        out = np.zeros((na, n_envs, 2), dtype=np.float32)
        oobs = np.zeros((na, n_envs, self.cfg.obs_dim), dtype=np.float32) if return_obs else None
        check(self.lib.fqlpop_rollout(self._h, fptr(obs), n_envs, int(max_steps),
                                      ctypes.c_uint64(int(seed) & (2**64 - 1)),
                                      None if nz is None else fptr(nz), fptr(out),
                                      None if oobs is None else fptr(oobs)))
        if return_obs:
            return out[..., 0], out[..., 1], oobs
        return out[..., 0], out[..., 1]

    def envmodel_step(self, observations, actions):
        """One state-predictor + termination-predictor step on the GPU:
        returns (next_observations [n, obs], termination logits [n])."""
        obs = _f32(observations).reshape(-1, self.cfg.obs_dim)
        act = _f32(actions).reshape(-1, self.cfg.action_dim)
        n = obs.shape[0]
        if act.shape[0] != n:
            raise ValueError("observations and actions differ in rows")
        nxt = np.zeros_like(obs)
        logit = np.zeros(n, dtype=np.float32)
        check(self.lib.fqlpop_envmodel_step(self._h, fptr(obs), fptr(act), n, fptr(nxt), fptr(logit)))
        return nxt, logit

    # ----------------------------------------------------------------- state
    def get_flat(self, member: int, which: int = STATE_PARAMS) -> np.ndarray:
        flat = np.zeros(self.state_size, dtype=np.float32)
        check(self.lib.fqlpop_get_state(self._h, int(member), int(which), fptr(flat), self.state_size))
        return flat

    def set_flat(self, member: int, flat, which: int = STATE_PARAMS):
        flat = _f32(flat).reshape(-1)
        if flat.shape[0] != self.state_size:
            raise ValueError("flat state size mismatch")
        check(self.lib.fqlpop_set_state(self._h, int(member), int(which), fptr(flat), self.state_size))

    def flat_to_tree(self, flat) -> dict:
        """Flat state -> {net: {"Dense_0/kernel": array, ...}} (oracle naming)."""
        tree = {}
        for name, off, shape in self.leaves:
            net, leaf = name.split("/", 1)
            size = int(np.prod(shape))
            tree.setdefault(net, {})[leaf] = np.asarray(flat[off:off + size]).reshape(shape).copy()
        return tree

    def tree_to_flat(self, tree) -> np.ndarray:
        flat = np.zeros(self.state_size, dtype=np.float32)
        for name, off, shape in self.leaves:
            net, leaf = name.split("/", 1)
            arr = np.asarray(tree[net][leaf], dtype=np.float32)
            if arr.shape != shape:
                raise ValueError(f"{name}: shape {arr.shape} != {shape}")
            flat[off:off + arr.size] = arr.reshape(-1)
        return flat

    def get_params(self, member: int) -> dict:
        return self.flat_to_tree(self.get_flat(member, STATE_PARAMS))

    def set_params(self, member: int, tree: dict):
        self.set_flat(member, self.tree_to_flat(tree), STATE_PARAMS)

    def get_count(self, member: int) -> int:
        c = ctypes.c_int32()
        check(self.lib.fqlpop_get_count(self._h, int(member), ctypes.byref(c)))
        return int(c.value)

    def set_count(self, member: int, count: int):
        check(self.lib.fqlpop_set_count(self._h, int(member), int(count)))

    def set_member(self, member: int, alpha: float, seed: int, reinit: bool = True):
        check(self.lib.fqlpop_set_member(self._h, int(member), float(alpha),
                                         ctypes.c_uint64(int(seed) & (2**64 - 1)), int(bool(reinit))))
        self.alphas[member] = alpha
        self.seeds[member] = seed

    def state_dict(self, member: int) -> dict:
        """Member state in flax ``to_state_dict`` shape: params (incl. target
        critic), Adam (count, mu, nu) -- names follow oracle/fql_oracle.py."""
        return {"params": self.get_params(member),
                "opt_state": {"count": self.get_count(member),
                              "mu": self.flat_to_tree(self.get_flat(member, STATE_ADAM_M)),
                              "nu": self.flat_to_tree(self.get_flat(member, STATE_ADAM_V))},
                "alpha": float(self.alphas[member]), "seed": int(self.seeds[member])}

    def load_state_dict(self, member: int, sd: dict):
        self.set_params(member, sd["params"])
        self.set_flat(member, self.tree_to_flat(sd["opt_state"]["mu"]), STATE_ADAM_M)
        self.set_flat(member, self.tree_to_flat(sd["opt_state"]["nu"]), STATE_ADAM_V)
        self.set_count(member, int(sd["opt_state"]["count"]))

    def set_probe(self, enable: bool = True):
        check(self.lib.fqlpop_set_probe(self._h, int(bool(enable))))

    def read_probe(self):
        """(mean duration in us, launches, (event_us, stamp_us)) of the dominant
        kernel inside step(); the pair is the last clock cross-check."""
        tot = ctypes.c_double()
        n = ctypes.c_int64()
        cc = (ctypes.c_double * 2)()
        check(self.lib.fqlpop_read_probe(self._h, ctypes.byref(tot), ctypes.byref(n), cc))
        mean = tot.value / n.value if n.value else float("nan")
        return mean, int(n.value), (float(cc[0]), float(cc[1]))

    def probe_coverage(self):
        """(blocks stamped, blocks launched) over the probed launches since set_probe."""
        seen, exp = ctypes.c_int64(), ctypes.c_int64()
        check(self.lib.fqlpop_probe_coverage(self._h, ctypes.byref(seen), ctypes.byref(exp)))
        return int(seen.value), int(exp.value)

    def dominant_kernel_info(self):
        """(kernel symbol, algorithmic FLOPs, unique HBM bytes) of one launch of
        the step's dominant kernel over the active members."""
        name = ctypes.create_string_buffer(128)
        fl = ctypes.c_double()
        by = ctypes.c_double()
        check(self.lib.fqlpop_dominant_kernel_info(self._h, name, 128, ctypes.byref(fl), ctypes.byref(by)))
        return name.value.decode(), float(fl.value), float(by.value)

    def dominant_kernel_flops(self) -> float:
        """Algorithmic FLOPs of one dominant-kernel launch (all active members)."""
        return self.dominant_kernel_info()[1]

    def time_dominant_kernel(self, iters: int = 50):
        us = ctypes.c_double()
        fl = ctypes.c_double()
        check(self.lib.fqlpop_time_dominant_kernel(self._h, int(iters), ctypes.byref(us), ctypes.byref(fl)))
        return float(us.value), float(fl.value)
