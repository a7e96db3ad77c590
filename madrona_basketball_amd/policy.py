"""Fused policy inference: the reference's Agent
(scripts/agent.py:108-154, 32 channels, 2 layers, buckets [2,8,3,2,2,2]) run
by one gfx950 kernel (bb_policy_forward, csrc/bb_policy.hip) that writes its
actions straight into the simulator's action tensor -- the
`actions, log_probs, values = agent(obs)` + `actions[:, i] = a` pair of
scripts/ppo.py:67 / scripts/env.py:147 without a round trip through torch.

FusedPolicy.from_agent(agent) snapshots the weights of any torch module with
the reference Agent's layout (obs_norm.mean/var, backbone Linear/LayerNorm,
actor, critic); call refresh() after an optimizer step.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .madrona import ExecMode

BUCKETS = (2, 8, 3, 2, 2, 2)
IN, HID, LOGITS, HEAD = 128, 32, 19, 32


class _ObsNorm(torch.nn.Module):
    """RunningMeanStd's state (scripts/agent.py:19-26): float64 mean / var, eps."""

    def __init__(self, dim: int):
        super().__init__()
        self.epsilon = 1e-5
        self.register_buffer("mean", torch.zeros(dim, dtype=torch.float64))
        self.register_buffer("var", torch.ones(dim, dtype=torch.float64))


def make_agent(seed: int = 0) -> torch.nn.Module:
    """A torch module with the reference Agent's layout and initialisation
    (scripts/agent.py:97-131: Kaiming-normal backbone, orthogonal heads at gain
    0.01, zero biases, identity observation normaliser) -- random weights of
    that architecture for benchmarks and tests (no checkpoints here)."""
    g = torch.Generator().manual_seed(seed)
    m = torch.nn.Module()
    m.action_buckets = list(BUCKETS)
    m.backbone = torch.nn.Sequential(torch.nn.Linear(IN, HID), torch.nn.LayerNorm(HID), torch.nn.ReLU(),
                                     torch.nn.Linear(HID, HID), torch.nn.LayerNorm(HID), torch.nn.ReLU())
    m.actor = torch.nn.Linear(HID, LOGITS)
    m.critic = torch.nn.Linear(HID, 1)
    m.obs_norm = _ObsNorm(IN)
    with torch.no_grad():
        for lin in (m.backbone[0], m.backbone[3]):
            torch.nn.init.kaiming_normal_(lin.weight, torch.nn.init.calculate_gain("relu"), generator=g)
            lin.bias.zero_()
        for lin in (m.actor, m.critic):
            torch.nn.init.orthogonal_(lin.weight, gain=0.01, generator=g)
            lin.bias.zero_()
    return m


def agent_from_state_dict(state_dict: dict, device=None) -> torch.nn.Module:
    """A module of the reference Agent's layout holding `state_dict` -- the
    keys Agent.state_dict() / a checkpoint written by scripts/ppo.py has
    (backbone.{0,1,3,4}.*, actor.*, critic.*, obs_norm.mean/var; the
    value_norm / count buffers are not used by inference).  Load checkpoints
    with torch.load(path, weights_only=True), as Agent.load does
    (scripts/agent.py:180-182)."""
    m = make_agent(0)
    own = m.state_dict()
    missing = [k for k in own if k not in state_dict]
    if missing:
        raise KeyError(f"state_dict lacks {missing}")
    with torch.no_grad():
        for k, v in own.items():
            src = torch.as_tensor(state_dict[k])
            if tuple(src.shape) != tuple(v.shape):
                raise ValueError(f"{k}: shape {tuple(src.shape)}, expected {tuple(v.shape)}")
            v.copy_(src.to(v.dtype))
    return m if device is None else m.to(device)


class FusedPolicy:
    def __init__(self, device: torch.device):
        self.device = torch.device(device)
        self._tensors = {}

    @classmethod
    def from_agent(cls, agent, device=None) -> "FusedPolicy":
        dev = device or next(agent.parameters()).device
        p = cls(dev)
        p.agent = agent
        p.refresh()
        return p

    @torch.no_grad()
    def refresh(self) -> None:
        """Re-read the agent's weights (after an update)."""
        a = self.agent
        lin = [m for m in a.backbone if isinstance(m, torch.nn.Linear)]
        lns = [m for m in a.backbone if isinstance(m, torch.nn.LayerNorm)]
        if (len(lin) != 2 or lin[0].in_features != IN or lin[0].out_features != HID or lin[1].out_features != HID
                or a.actor.out_features != LOGITS or tuple(a.action_buckets) != BUCKETS):
            raise ValueError("FusedPolicy supports the reference configuration: input 128, num_channels 32, "
                             "num_layers 2, buckets [2, 8, 3, 2, 2, 2] (scripts/env.py:107)")
        dev, f32 = self.device, torch.float32

        def t(x):
            return x.detach().to(device=dev, dtype=f32).contiguous()
        # RunningMeanStd.forward (agent.py:29-35): mean/var cast to f32, var + eps, rsqrt
        mean = a.obs_norm.mean.to(f32)
        var = a.obs_norm.var.to(f32) + a.obs_norm.epsilon
        head_w = torch.zeros((HEAD, HID), dtype=f32, device=dev)
        head_b = torch.zeros((HEAD,), dtype=f32, device=dev)
        head_w[:LOGITS] = t(a.actor.weight)
        head_w[LOGITS] = t(a.critic.weight)[0]
        head_b[:LOGITS] = t(a.actor.bias)
        head_b[LOGITS] = t(a.critic.bias)[0]
        self._tensors = {
            "obs_mean": t(mean), "obs_inv": t(torch.rsqrt(var.to(dev))),
            "w1": t(lin[0].weight), "b1": t(lin[0].bias), "ln1_w": t(lns[0].weight), "ln1_b": t(lns[0].bias),
            "w2": t(lin[1].weight), "b2": t(lin[1].bias), "ln2_w": t(lns[1].weight), "ln2_b": t(lns[1].bias),
            "head_w": head_w, "head_b": head_b,
        }
        self._w = _lib.PolicyWeights(**{k: v.data_ptr() for k, v in self._tensors.items()})

    def to(self, device) -> "FusedPolicy":
        """A copy of the packed weights on another device (same bits)."""
        p = FusedPolicy(device)
        p.agent = getattr(self, "agent", None)
        p._tensors = {k: v.to(p.device).contiguous() for k, v in self._tensors.items()}
        p._w = _lib.PolicyWeights(**{k: v.data_ptr() for k, v in p._tensors.items()})
        return p

    def _stream(self):
        if self.device.type == "cuda":
            return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        return ctypes.c_void_p(None)

    def forward_into(self, obs: torch.Tensor, actions: torch.Tensor, log_prob: torch.Tensor = None,
                     value: torch.Tensor = None, stochastic: bool = True, seed: int = 0, step: int = 0) -> None:
        """obs [R, >=128] float32 rows (any row stride, e.g. obs_tensor[:, agent]);
        actions [R, 6] int32 rows (any row stride, e.g. action_tensor[:, agent])."""
        rows = obs.shape[0]
        if obs.dim() != 2 or obs.shape[1] < IN or obs.stride(1) != 1 or obs.dtype != torch.float32:
            raise ValueError("obs must be float32 [rows, >=128] with unit column stride")
        if (actions.dim() != 2 or actions.shape != (rows, 6) or actions.stride(1) != 1
                or actions.dtype != torch.int32):
            raise ValueError("actions must be int32 [rows, 6] with unit column stride")
        for t in (obs, actions, log_prob, value):
            if t is not None and t.device != self.device:
                raise ValueError("all tensors must live on the policy's device")
        for t in (log_prob, value):
            if t is not None and (t.shape != (rows,) or not t.is_contiguous() or t.dtype != torch.float32):
                raise ValueError("log_prob / value must be contiguous float32 [rows]")
        mode = ExecMode.CUDA if self.device.type == "cuda" else ExecMode.CPU
        _lib.check(_lib.load().bb_policy_forward(
            ctypes.byref(self._w), int(mode), self.device.index if self.device.index is not None else -1,
            ctypes.c_void_p(obs.data_ptr()), rows, obs.stride(0), ctypes.c_void_p(actions.data_ptr()),
            actions.stride(0), ctypes.c_void_p(None if log_prob is None else log_prob.data_ptr()),
            ctypes.c_void_p(None if value is None else value.data_ptr()), 1 if stochastic else 0,
            int(seed) & 0xFFFFFFFF, int(step) & 0xFFFFFFFF, self._stream()), "policy_forward")

    def __call__(self, obs: torch.Tensor, stochastic: bool = True, seed: int = 0, step: int = 0):
        """Agent.forward's outputs (actions int32 [R, 6], log_probs [R], values [R])."""
        rows = obs.shape[0]
        actions = torch.empty((rows, 6), dtype=torch.int32, device=self.device)
        lp = torch.empty((rows,), dtype=torch.float32, device=self.device)
        v = torch.empty((rows,), dtype=torch.float32, device=self.device)
        self.forward_into(obs, actions, lp, v, stochastic, seed, step)
        return actions, lp, v

    def act(self, sim, agent_idx: int, log_prob: torch.Tensor = None, value: torch.Tensor = None,
            stochastic: bool = True, seed: int = 0, step: int = 0) -> None:
        """Observe agent `agent_idx` of every world and write its actions into the
        simulator's action tensor (env.py:147's `actions[:, i] = a`), on the device."""
        obs = sim.observations_tensor().to_torch()[:, agent_idx]
        act = sim.action_tensor().to_torch()[:, agent_idx]
        self.forward_into(obs, act, log_prob, value, stochastic, seed, step)

    # ------------------------------------------------------------ PPO rollout
    ROLLOUT_KEYS = ("obs", "actions", "log_prob", "value", "reward", "done", "next_value")

    def rollout_buffers(self, sim, n: int) -> dict:
        """Zeroed outputs of rollout() on the simulator's device -- the storage of
        scripts/buffers.py:4-11 for n steps of the trainee (obs [n, W, 128],
        actions int32 [n, W, 6], log_prob / value / reward / done [n, W]) and
        next_value [W] (ppo.py:136-137)."""
        W, dev, f32 = sim.num_worlds, sim.device, torch.float32
        return {"obs": torch.zeros((n, W, IN), dtype=f32, device=dev),
                "actions": torch.zeros((n, W, 6), dtype=torch.int32, device=dev),
                "log_prob": torch.zeros((n, W), dtype=f32, device=dev),
                "value": torch.zeros((n, W), dtype=f32, device=dev),
                "reward": torch.zeros((n, W), dtype=f32, device=dev),
                "done": torch.zeros((n, W), dtype=f32, device=dev),
                "next_value": torch.zeros((W,), dtype=f32, device=dev)}

    def rollout(self, sim, n: int, buffers: dict, trainee: int = 0, stochastic: bool = True, seed: int = 0,
                step0: int = 0, opponent: "FusedPolicy" = None, per_step: bool = False, time_kernels: bool = False):
        """PPO's rollout loop (scripts/ppo.py:61-141) on the device, bb_rollout_policy:
        n x (this policy acts for agent `trainee` of every world; [the frozen
        `opponent` acts for the other agent, env.py:127-143]; step) with the
        buffer stores of ppo.py:129-134 and next_value = evaluate(last obs).
        Bit for bit n x (act(); [opponent.act()]; sim.step()) with the same reads.
        Any entry of `buffers` may be None (not recorded).  On gfx950 (2 agents,
        no opponent, up to 16 384 worlds) one fused launch runs every step;
        per_step=True forces a policy launch + a step launch per step.  Returns
        the elapsed device ms when time_kernels."""
        W = sim.num_worlds
        shapes = {"obs": ((n, W, IN), torch.float32), "actions": ((n, W, 6), torch.int32),
                  "log_prob": ((n, W), torch.float32), "value": ((n, W), torch.float32),
                  "reward": ((n, W), torch.float32), "done": ((n, W), torch.float32),
                  "next_value": ((W,), torch.float32)}
        ptrs = {}
        for k in self.ROLLOUT_KEYS:
            t = buffers.get(k)
            if t is not None:
                shp, dt = shapes[k]
                if tuple(t.shape) != shp or t.dtype != dt or not t.is_contiguous() or t.device != sim.device:
                    raise ValueError(f"rollout buffer {k!r} must be a contiguous {dt} {shp} tensor on the "
                                     "simulator's device")
            ptrs[k] = None if t is None else t.data_ptr()
        if (buffers.get("reward") is None) != (buffers.get("done") is None):
            raise ValueError("reward and done are recorded together")
        if sim.device != self.device or (opponent is not None and opponent.device != self.device):
            raise ValueError("policy, opponent and simulator must share a device")
        out = _lib.PolicyRolloutBuffers(**ptrs)
        ms = ctypes.c_float(0.0)
        _lib.check(_lib.load().bb_rollout_policy(
            sim._h, ctypes.byref(self._w), ctypes.byref(opponent._w) if opponent is not None else None, int(n),
            int(trainee), 1 if stochastic else 0, int(seed) & 0xFFFFFFFF, int(step0) & 0xFFFFFFFF,
            ctypes.byref(out), _lib.ROLLOUT_PER_STEP if per_step else 0, sim._stream(),
            ctypes.byref(ms) if time_kernels else None), "rollout_policy")
        return ms.value if time_kernels else None
