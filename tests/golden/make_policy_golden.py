"""Generate tests/golden/policy_golden.npz from the reference's own Agent.

Run in the build container (where /root/reference exists):
    python tests/golden/make_policy_golden.py

The reference modules scripts/agent.py, scripts/action.py and
scripts/moving_avg.py import only torch, so they are imported here, from
/root/reference, and nothing of them is copied: the fixture holds data only
(weights, observation rows, outputs).  The reference never travels to the GPU
box; tests/test_policy_golden.py reads the .npz.

Cases (both on the same observation rows, produced by the oracle -- the
product's checker -- from the reference's env.py workload shape):
  * "init":   Agent(128, 32, 2, [2, 8, 3, 2, 2, 2]) exactly as
              scripts/agent.py:108-131 initialises it under torch.manual_seed,
              its RunningMeanStd updated with the rows by the reference's own
              update() (scripts/agent.py:40-50, what ppo.py does each rollout);
  * "scaled": the same module with the actor / critic heads and their biases
              scaled as training would (the orthogonal gain-0.01 heads give
              logits of ~1e-2, where argmax margins are tiny).

Outputs recorded per case, all computed by the reference code:
  logits  = agent.actor(agent.norm_obs_backbone(obs))         (agent.py:134-144)
  best    = DiscreteActionDistributions(buckets, logits).best() (action.py:21-23)
  logp    = action_stats(best)[0].sum(-1)   (action.py:36-44; see note)
  value   = agent.critic(x).squeeze(-1)                        (agent.py:153)
Note: Agent.forward(stochastic=False) pairs the 6 distributions with the
first 6 *rows* of the action tensor (action.py:25-27 zips over rows), which
only broadcasts for 1 or 6 rows; the per-column log-prob of the best actions
is action_stats', which is what the fused policy returns.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

REF_SCRIPTS = "/root/reference/scripts"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "policy_golden.npz")
BUCKETS = [2, 8, 3, 2, 2, 2]
SEED = 20261016
# The reference modules this script imports (and so executes), pinned to the
# contents they had when policy_golden.npz was generated: a changed file is
# refused rather than run.
REF_SHA256 = {
    "agent.py": "8215be664e07b131f8751428bffe0c2ec0801bdc3d2214a82d8b4c1685bff67e",
    "action.py": "b1511f622fb76412bc9ec869c22f3891f94ea06b90710e9add49e5ed9ad156e8",
    "moving_avg.py": "dfe803c863899f22162fcdbd86930506563e8e1c6d0f1873e26d886911c8c966",
}


def check_reference_files() -> None:
    import hashlib
    for name, want in REF_SHA256.items():
        with open(os.path.join(REF_SCRIPTS, name), "rb") as f:
            got = hashlib.sha256(f.read()).hexdigest()
        if got != want:
            raise SystemExit(f"refusing to import {REF_SCRIPTS}/{name}: sha256 {got} != pinned {want}")


def observation_rows(worlds: int = 256, steps: int = 150) -> np.ndarray:
    """[2 * worlds, 128] float32: both agents' rows after `steps` random steps."""
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    o = O.Oracle(worlds, num_agents=2, flags=O.FLAG_PER_WORLD_RNG)
    o.run_random(steps, 321, 0)
    return np.ascontiguousarray(o.export("observations").reshape(-1, 128).astype(np.float32))


def main():
    obs_np = observation_rows()
    check_reference_files()
    sys.path.insert(0, REF_SCRIPTS)
    from action import DiscreteActionDistributions  # noqa: E402  (reference module)
    from agent import Agent  # noqa: E402  (reference module)

    torch.manual_seed(SEED)
    agent = Agent(128, 32, 2, BUCKETS)
    obs = torch.from_numpy(obs_np)
    agent.update_obs_normalizer(obs)  # the reference's RunningMeanStd.update

    out = {"obs": obs_np, "buckets": np.array(BUCKETS, dtype=np.int32)}

    def record(name: str):
        with torch.no_grad():
            x = agent.norm_obs_backbone(obs)
            logits = agent.actor(x)
            dists = DiscreteActionDistributions(BUCKETS, logits=logits)
            best = dists.best()
            logp, _ = dists.action_stats(best)
            value = agent.critic(x).squeeze(-1)
        for k, v in agent.state_dict().items():
            out[f"{name}/w/{k}"] = v.detach().cpu().numpy().copy()  # not a view of the live parameter
        out[f"{name}/logits"] = logits.numpy().astype(np.float32)
        out[f"{name}/best"] = best.numpy().astype(np.int32)
        out[f"{name}/logp"] = logp.sum(-1).numpy().astype(np.float32)
        out[f"{name}/value"] = value.numpy().astype(np.float32)

    record("init")
    g = torch.Generator().manual_seed(SEED + 1)
    with torch.no_grad():
        agent.actor.weight.mul_(150.0)
        agent.critic.weight.mul_(150.0)
        agent.actor.bias.copy_(torch.randn(agent.actor.bias.shape, generator=g) * 0.5)
        agent.critic.bias.copy_(torch.randn(agent.critic.bias.shape, generator=g) * 0.5)
    record("scaled")
    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT}: {len(out)} arrays, {os.path.getsize(OUT)} bytes")


if __name__ == "__main__":
    main()
