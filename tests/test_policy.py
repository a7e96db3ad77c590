"""Fused policy inference (bb_policy_forward).

The checker is a plain torch fp32 restatement of the reference's Agent
(scripts/agent.py:19-38 RunningMeanStd, :108-154 Agent; scripts/action.py
Categorical buckets) -- test infrastructure, built here from its published
structure.  Bars: host executor == gfx950 kernel bit for bit (same arithmetic
order, bb_policy.h); both vs the torch restatement within fp32 tolerance
(value / log-prob |diff| <= 2e-5 + 2e-5 |x|, written in the test), argmax
actions equal wherever the top two logits of a bucket are > 1e-4 apart;
inverse-CDF samples follow softmax(logits) (binomial 5-sigma bounds).
"""
import numpy as np
import pytest
import torch
import torch.nn as nn

from madrona_basketball_amd import ExecMode
from madrona_basketball_amd.policy import BUCKETS, FusedPolicy
from tests.helpers import make_sim

TOL_ABS, TOL_REL = 2e-5, 2e-5


class RunningMeanStd(nn.Module):  # scripts/agent.py:19-38 (forward only)
    def __init__(self, dim, clamp=5.0):
        super().__init__()
        self.epsilon, self.clamp = 1e-5, clamp
        self.register_buffer("mean", torch.zeros(dim, dtype=torch.float64))
        self.register_buffer("var", torch.ones(dim, dtype=torch.float64))

    def forward(self, x):
        mean = self.mean.to(torch.float32)
        var = self.var.to(torch.float32) + self.epsilon
        return torch.clamp((x - mean) * torch.rsqrt(var), min=-self.clamp, max=self.clamp)


class RefAgent(nn.Module):  # scripts/agent.py:108-154 at num_channels 32, num_layers 2
    def __init__(self, seed=0):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.action_buckets = list(BUCKETS)
        self.backbone = nn.Sequential(nn.Linear(128, 32), nn.LayerNorm(32), nn.ReLU(),
                                      nn.Linear(32, 32), nn.LayerNorm(32), nn.ReLU())
        self.actor = nn.Linear(32, 19)
        self.critic = nn.Linear(32, 1)
        self.obs_norm = RunningMeanStd(128)
        with torch.no_grad():
            for p in self.parameters():
                p.copy_(torch.randn(p.shape, generator=g) * (0.5 if p.dim() > 1 else 0.3))
            self.obs_norm.mean.copy_(torch.randn(128, generator=g, dtype=torch.float64) * 3)
            self.obs_norm.var.copy_(torch.rand(128, generator=g, dtype=torch.float64) * 20 + 0.01)

    def logits_value(self, obs):
        x = self.backbone(self.obs_norm(obs))
        return self.actor(x), self.critic(x).squeeze(-1)

    def forward_best(self, obs):
        logits, value = self.logits_value(obs)
        acts, lps, o = [], [], 0
        for nb in BUCKETS:
            sl = logits[:, o:o + nb]
            d = torch.distributions.Categorical(logits=sl, validate_args=False)
            a = d.probs.argmax(dim=-1)
            acts.append(a)
            lps.append(d.log_prob(a))
            o += nb
        return torch.stack(acts, 1), torch.stack(lps, 1).sum(-1), value, logits


def real_obs(mode, W=4096, steps=150):
    sim = make_sim(mode, W, per_world_rng=True)
    sim.step_n(steps, random_actions=True, action_seed=12)
    return sim, sim.observations_tensor().to_torch()


def margin_ok(logits):
    """Rows whose argmax is unambiguous in every bucket (top-2 gap > 1e-4)."""
    ok, o = torch.ones(logits.shape[0], dtype=torch.bool, device=logits.device), 0
    for nb in BUCKETS:
        top = torch.topk(logits[:, o:o + nb], 2, dim=-1).values
        ok &= (top[:, 0] - top[:, 1]) > 1e-4
        o += nb
    return ok


def check_vs_torch(ref, obs, acts, lp, v):
    ra, rlp, rv, logits = ref.forward_best(obs)
    assert torch.all((v - rv).abs() <= TOL_ABS + TOL_REL * rv.abs()), (v - rv).abs().max()
    assert torch.all((lp - rlp).abs() <= TOL_ABS + TOL_REL * rlp.abs()), (lp - rlp).abs().max()
    ok = margin_ok(logits)
    assert ok.float().mean() > 0.95
    assert torch.equal(acts[ok].long(), ra[ok])


@pytest.mark.parametrize("agent_idx", [0, 1])
def test_host_policy_vs_torch(native_lib, agent_idx):
    sim, obs_all = real_obs(ExecMode.CPU, W=1024, steps=120)
    ref = RefAgent(seed=3)
    pol = FusedPolicy.from_agent(ref)
    obs = obs_all[:, agent_idx]
    acts, lp, v = pol(obs, stochastic=False)
    with torch.no_grad():
        check_vs_torch(ref, obs, acts, lp, v)


def test_host_policy_act_writes_one_agent_column(native_lib):
    sim, obs_all = real_obs(ExecMode.CPU, W=256, steps=50)
    ref = RefAgent(seed=4)
    pol = FusedPolicy.from_agent(ref)
    before = sim.action_tensor().to_torch().clone()
    lp = torch.empty(256)
    v = torch.empty(256)
    pol.act(sim, 1, lp, v, stochastic=False)
    after = sim.action_tensor().to_torch()
    assert torch.equal(after[:, 0], before[:, 0])
    a, lp2, v2 = pol(obs_all[:, 1], stochastic=False)
    assert torch.equal(after[:, 1], a) and torch.equal(lp, lp2) and torch.equal(v, v2)
    hi = torch.tensor(BUCKETS, dtype=torch.int32)
    assert torch.all((after[:, 1] >= 0) & (after[:, 1] < hi))


def test_host_policy_sampling_follows_softmax(native_lib):
    """20 000 copies of one observation row: per-bucket sample frequencies
    match softmax(logits) within 5 binomial sigma; log-probs are those of the
    sampled actions."""
    ref = RefAgent(seed=5)
    with torch.no_grad():
        ref.actor.weight.mul_(0.05)  # keep every class's probability sizeable
    pol = FusedPolicy.from_agent(ref)
    _, obs_all = real_obs(ExecMode.CPU, W=8, steps=30)
    R = 20000
    obs = obs_all[3, 0].repeat(R, 1).contiguous()
    acts, lp, _ = pol(obs, stochastic=True, seed=7, step=1)
    with torch.no_grad():
        logits, _ = ref.logits_value(obs[:1])
    o = 0
    exp_lp = torch.zeros(R)
    for b, nb in enumerate(BUCKETS):
        p = torch.softmax(logits[0, o:o + nb], -1)
        freq = torch.bincount(acts[:, b].long(), minlength=nb).float() / R
        sigma = torch.sqrt(p * (1 - p) / R)
        assert torch.all((freq - p).abs() <= 5 * sigma + 1e-6), (b, freq, p)
        exp_lp += torch.log_softmax(logits[0, o:o + nb], -1)[acts[:, b].long()]
        o += nb
    assert torch.allclose(lp, exp_lp, atol=1e-4)
    a2, _, _ = pol(obs, stochastic=True, seed=7, step=2)
    assert not torch.equal(acts, a2)  # the step is part of the key


@pytest.mark.gpu
@pytest.mark.parametrize("stochastic", [False, True])
def test_gpu_policy_equals_host_and_torch(native_lib, stochastic):
    assert torch.cuda.is_available()
    sim, obs_all = real_obs(ExecMode.CUDA, W=65536, steps=150)
    ref = RefAgent(seed=9).cuda()
    pol_g = FusedPolicy.from_agent(ref)           # device
    pol_h = pol_g.to("cpu")                       # the same packed bits on the host
    obs = obs_all[:, 0]
    ag, lpg, vg = pol_g(obs, stochastic=stochastic, seed=3, step=11)
    ah, lph, vh = pol_h(obs.cpu(), stochastic=stochastic, seed=3, step=11)
    torch.cuda.synchronize()
    assert torch.equal(ag.cpu(), ah)
    assert torch.equal(lpg.cpu().view(torch.int32), lph.view(torch.int32))
    assert torch.equal(vg.cpu().view(torch.int32), vh.view(torch.int32))
    if not stochastic:
        with torch.no_grad():
            check_vs_torch(ref, obs, ag, lpg, vg)


@pytest.mark.gpu
def test_gpu_policy_multi_tile_waves_equal_host(native_lib):
    """Every agent's rows (131 072 > 1 024 tiles of 64): each persistent wave
    runs two tiles, the second tile's rows loaded under the first's network;
    bit-identical to the host policy."""
    assert torch.cuda.is_available()
    sim, obs_all = real_obs(ExecMode.CUDA, W=65536, steps=60)
    pol_g = FusedPolicy.from_agent(RefAgent(seed=4).cuda())
    pol_h = pol_g.to("cpu")
    obs = obs_all.reshape(-1, obs_all.shape[-1])
    for stochastic in (False, True):
        ag, lpg, vg = pol_g(obs, stochastic=stochastic, seed=5, step=3)
        ah, lph, vh = pol_h(obs.cpu(), stochastic=stochastic, seed=5, step=3)
        torch.cuda.synchronize()
        assert torch.equal(ag.cpu(), ah)
        assert torch.equal(lpg.cpu().view(torch.int32), lph.view(torch.int32))
        assert torch.equal(vg.cpu().view(torch.int32), vh.view(torch.int32))


@pytest.mark.gpu
def test_gpu_policy_act_in_the_loop(native_lib):
    """env.py's loop with the fused policy writing the trainee's actions:
    device run == host run of the same loop, bit for bit."""
    assert torch.cuda.is_available()
    pol_g = FusedPolicy.from_agent(RefAgent(seed=2).cuda())
    pol_h = pol_g.to("cpu")
    g = make_sim(ExecMode.CUDA, 2048, per_world_rng=True)
    h = make_sim(ExecMode.CPU, 2048, per_world_rng=True)
    for t in range(200):
        pol_g.act(g, 0, stochastic=True, seed=1, step=t)
        pol_h.act(h, 0, stochastic=True, seed=1, step=t)
        g.step()
        h.step()
    torch.cuda.synchronize()
    for name in g._views:
        assert torch.equal(g._views[name].cpu(), h._views[name]), name
