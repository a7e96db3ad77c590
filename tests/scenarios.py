"""Scripted scenarios that force the rare paths of the reference rules.

Actions are computed from the oracle's state and fed identically to the
simulator under test, so the same script drives both sides in lockstep.
"""
from __future__ import annotations

import math

import numpy as np


def steer(frm, to) -> int:
    """moveAngle k moves along (sin(k pi/4), -cos(k pi/4)) (game.cpp:432-435)."""
    d = np.asarray(to, np.float64) - np.asarray(frm, np.float64)
    return int(round(math.atan2(d[0], -d[1]) / (math.pi / 4))) % 8


class FullGameInbound:
    """isOneOnOne = 0, tag override off, defender idle: walk to the loose ball,
    grab it, shoot it out of bounds -> inbound to the other team
    (game.cpp:1083-1111) -> 5 s inbound violation turnover (game.cpp:1116-1157)
    -> pass (game.cpp:243-270) -> out of bounds again ...  Expected events
    are asserted by the callers."""

    def __init__(self, num_worlds: int, num_agents: int = 2):
        self.W = num_worlds
        self.N = num_agents
        self.phase = np.zeros(num_worlds, np.int32)

    def prepare(self, oracle, sim_attr_tensor=None):
        at = oracle.export("attributes")
        at[:, 1:, 4] = 0.0  # reaction speed 0 for all but agent 0: no chase, no tags
        oracle.import_("attributes", at)
        if sim_attr_tensor is not None:
            import torch
            sim_attr_tensor.copy_(torch.from_numpy(at).to(sim_attr_tensor.device))

    def actions(self, oracle, t: int) -> np.ndarray:
        a = np.zeros((self.W, self.N, 6), np.int32)
        pos = oracle.export("agent_pos")
        ball = oracle.export("ball_pos")[:, 0]
        poss = oracle.export("agent_possession")
        for w in range(self.W):
            if self.phase[w] == 0:
                if np.linalg.norm(ball[w, :2] - pos[w, 0, :2]) > 0.25:
                    a[w, 0, 0] = 1
                    a[w, 0, 1] = steer(pos[w, 0, :2], ball[w, :2])
                else:
                    a[w, 0, 3] = 1
                    self.phase[w] = 1
            elif self.phase[w] == 1:
                if poss[w, 0, 0] == 1:
                    a[w, 0, 2] = 1 + (w % 2)   # some worlds turn while shooting
                    a[w, 0, 5] = 1
                    self.phase[w] = 2
            elif t > 600 + 7 * w:
                a[w, :, 4] = 1
        return a


class FullGameScore(FullGameInbound):
    """isOneOnOne = 0, tag override off, other agents idle: agent 0 walks to
    the loose ball, grabs it, carries it to within `shot_range` m of the hoop it
    attacks and shoots; a make takes the full-game branch of scoreSystem
    (game.cpp:905-950: score, ball to the baseline spot, assignInbounder to
    the team that was scored on), then the inbounder passes."""

    def __init__(self, num_worlds: int, num_agents: int = 2, shot_range: float = 1.2):
        super().__init__(num_worlds, num_agents)
        self.shot_range = shot_range

    def actions(self, oracle, t: int) -> np.ndarray:
        a = np.zeros((self.W, self.N, 6), np.int32)
        pos = oracle.export("agent_pos")
        ball = oracle.export("ball_pos")[:, 0]
        poss = oracle.export("agent_possession")
        hoops = oracle.export("hoop_pos")
        team = oracle.export("team")
        for w in range(self.W):
            # agent 0 attacks the hoop it does not defend (game.cpp:289-297)
            target = hoops[w, 1, :2] if team[w, 0, 4] == 0 else hoops[w, 0, :2]
            if self.phase[w] == 0:
                if np.linalg.norm(ball[w, :2] - pos[w, 0, :2]) > 0.25:
                    a[w, 0, 0] = 1
                    a[w, 0, 1] = steer(pos[w, 0, :2], ball[w, :2])
                else:
                    a[w, 0, 3] = 1
                    self.phase[w] = 1
            elif self.phase[w] == 1:
                if poss[w, 0, 0] == 1:
                    if np.linalg.norm(target - pos[w, 0, :2]) > self.shot_range:
                        a[w, 0, 0] = 1
                        a[w, 0, 1] = steer(pos[w, 0, :2], target)
                    else:
                        a[w, 0, 5] = 1
                        self.phase[w] = 2
            elif self.phase[w] == 2 and t % 40 == 0:
                a[w, :, 4] = 1  # the inbounder passes
        return a
