"""Fused policy vs fixtures produced by the reference's own Agent.

tests/golden/policy_golden.npz is written by tests/golden/make_policy_golden.py,
which imports scripts/agent.py / action.py from the reference (torch only) and
records, for 512 oracle observation rows and two weight sets ("init": the
reference initialisation with its RunningMeanStd updated on the rows;
"scaled": trained-like heads), the logits, best() actions, their summed
log-probs (action_stats) and the critic value.

Bars (fp32; the reference runs torch CPU fp32 GEMMs, the kernel an f32 MFMA
k-chain, so the sums round differently):
  value, log-prob:  |ours - ref| <= 2e-5 + 2e-5 |ref|
  actions:          equal in every bucket whose top-2 reference logits differ
                    by more than 1e-4 (an argmax closer than that is decided
                    by rounding); the rows left out are counted and bounded.
The host executor and the gfx950 kernel are also compared bit for bit.
"""
import os

import numpy as np
import pytest
import torch

from madrona_basketball_amd.policy import BUCKETS, FusedPolicy, agent_from_state_dict

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "policy_golden.npz")
TOL_ABS, TOL_REL, MARGIN = 2e-5, 2e-5, 1e-4
CASES = ["init", "scaled"]


def load_case(name):
    d = np.load(GOLDEN)  # allow_pickle=False (default): plain arrays
    sd = {k[len(name) + 3:]: torch.from_numpy(d[k]) for k in d.files if k.startswith(f"{name}/w/")}
    ref = {k: d[f"{name}/{k}"] for k in ("logits", "best", "logp", "value")}
    return torch.from_numpy(d["obs"]), sd, ref


def decisive(logits: np.ndarray) -> np.ndarray:
    """[rows, 6] bool: the bucket's argmax is decided by > MARGIN."""
    out, o = [], 0
    for nb in BUCKETS:
        s = np.sort(logits[:, o:o + nb], axis=1)
        out.append(s[:, -1] - s[:, -2] > MARGIN)
        o += nb
    return np.stack(out, 1)


def check(acts, lp, v, ref, min_decisive):
    acts, lp, v = acts.cpu().numpy(), lp.cpu().numpy(), v.cpu().numpy()
    assert np.all(np.abs(v - ref["value"]) <= TOL_ABS + TOL_REL * np.abs(ref["value"])), \
        np.abs(v - ref["value"]).max()
    assert np.all(np.abs(lp - ref["logp"]) <= TOL_ABS + TOL_REL * np.abs(ref["logp"])), \
        np.abs(lp - ref["logp"]).max()
    ok = decisive(ref["logits"])
    assert ok.mean() >= min_decisive, ok.mean()
    assert np.array_equal(acts[ok], ref["best"][ok])


MIN_DECISIVE = {"init": 0.5, "scaled": 0.99}


def test_golden_fixture_is_self_consistent():
    """The fixture's best() is the per-bucket argmax of its logits, and its
    log-probs are the log-softmax at those actions (plain numpy)."""
    for name in CASES:
        _, _, ref = load_case(name)
        lg = ref["logits"].astype(np.float64)
        o, lp = 0, np.zeros(lg.shape[0])
        for b, nb in enumerate(BUCKETS):
            s = lg[:, o:o + nb]
            assert np.array_equal(ref["best"][:, b], s.argmax(1))
            lse = np.log(np.exp(s - s.max(1, keepdims=True)).sum(1)) + s.max(1)
            lp += s[np.arange(len(s)), ref["best"][:, b]] - lse
            o += nb
        assert np.allclose(lp, ref["logp"], atol=1e-5)


@pytest.mark.parametrize("case", CASES)
def test_host_policy_matches_reference_agent(native_lib, case):
    obs, sd, ref = load_case(case)
    pol = FusedPolicy.from_agent(agent_from_state_dict(sd))
    acts, lp, v = pol(obs, stochastic=False)
    check(acts, lp, v, ref, MIN_DECISIVE[case])


@pytest.mark.parametrize("case", CASES)
def test_host_policy_sampled_logprob_matches_reference_logits(native_lib, case):
    """Sampled actions (inverse CDF): their log-probs are the reference's log-softmax at
    the sampled actions."""
    obs, sd, ref = load_case(case)
    pol = FusedPolicy.from_agent(agent_from_state_dict(sd))
    acts, lp, _ = pol(obs, stochastic=True, seed=9, step=4)
    lg = torch.from_numpy(ref["logits"]).double()
    exp_lp, o = torch.zeros(lg.shape[0], dtype=torch.float64), 0
    for b, nb in enumerate(BUCKETS):
        exp_lp += torch.log_softmax(lg[:, o:o + nb], -1).gather(1, acts[:, b:b + 1].long()).squeeze(1)
        o += nb
    assert torch.all((lp.double() - exp_lp).abs() <= 1e-4 + 1e-4 * exp_lp.abs())


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_gpu_policy_matches_reference_agent(native_lib, case):
    assert torch.cuda.is_available()
    obs, sd, ref = load_case(case)
    pol_g = FusedPolicy.from_agent(agent_from_state_dict(sd, "cuda"))
    pol_h = pol_g.to("cpu")
    for stochastic in (False, True):
        ag, lpg, vg = pol_g(obs.cuda(), stochastic=stochastic, seed=5, step=2)
        ah, lph, vh = pol_h(obs, stochastic=stochastic, seed=5, step=2)
        torch.cuda.synchronize()
        assert torch.equal(ag.cpu(), ah)
        assert torch.equal(lpg.cpu().view(torch.int32), lph.view(torch.int32))
        assert torch.equal(vg.cpu().view(torch.int32), vh.view(torch.int32))
        if not stochastic:
            check(ag, lpg, vg, ref, MIN_DECISIVE[case])
