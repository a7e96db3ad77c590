"""k_policy_wg (the policy's B operands in LDS, 12 waves per workgroup) forced
on at every row count (the policy_wg path override): ragged and small row
counts, argmax and sampling, plain and strided observation rows --
bit-identical to the host policy (bb_policy.h), as the register-weight kernel
is."""
import pytest


@pytest.mark.gpu
def test_gpu_policy_wg_forced_equals_host(native_lib):
    import torch
    from madrona_basketball_amd import ExecMode, _lib
    from madrona_basketball_amd.policy import FusedPolicy
    from tests.test_policy import RefAgent, real_obs
    sim, obs_all = real_obs(ExecMode.CUDA, W=70000, steps=40)
    pol_g = FusedPolicy.from_agent(RefAgent(seed=6).cuda())
    pol_h = pol_g.to("cpu")
    cases = [obs_all[:1, 0], obs_all[:17, 0], obs_all[:1000, 1], obs_all[:, 0],
             obs_all.reshape(-1, obs_all.shape[-1])[:40003]]
    with _lib.diag(policy_wg=1):
        for obs in cases:
            for stochastic in (False, True):
                ag, lpg, vg = pol_g(obs, stochastic=stochastic, seed=8, step=5)
                ah, lph, vh = pol_h(obs.cpu(), stochastic=stochastic, seed=8, step=5)
                torch.cuda.synchronize()
                assert torch.equal(ag.cpu(), ah), (obs.shape, stochastic)
                assert torch.equal(lpg.cpu().view(torch.int32), lph.view(torch.int32)), (obs.shape, stochastic)
                assert torch.equal(vg.cpu().view(torch.int32), vh.view(torch.int32)), (obs.shape, stochastic)
