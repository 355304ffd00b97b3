"""The reference's one-episode-per-update loop on the CPU oracle (test
infrastructure): fill_buffer! (utils.jl:389-402) and the body of train!
(utils.jl:434-481) / compute_D (compute_D.jl:89-138), taking the device's
counter-RNG decisions (tests/devrng.py) so a device run can be replayed
decision by decision. Parameters evolve on the oracle's own arithmetic
(fp64 gradient, Float32 RMSProp)."""
import numpy as np

import oracle
from devrng import explore, first_argmax, floyd


class OracleEpisodeLoop:
    def __init__(self, bs, C, cap, seed, th0, *, epsilon=1.0, decay=1e-6, epsilon_end=0.05, rate=1000,
                 batch=64, gamma=0.97):
        self.bs, self.C, self.cap, self.seed, self.B = bs, C, cap, seed, batch
        self.rate, self.decay, self.eps_end, self.gamma = rate, decay, epsilon_end, gamma
        self.eps = np.float32(epsilon)
        self.th = np.array(th0, np.float32, copy=True)
        self.acc = np.zeros_like(self.th)
        self.tt = self.th.copy()
        self.env = oracle.OracleBatch(1, bs, C)
        nc = bs * bs
        self.frames = np.zeros((cap, C + 1, nc), np.int8)
        self.act = np.zeros(cap, np.int32)
        self.rew = np.zeros(cap, np.float32)
        self.done = np.zeros(cap, np.uint8)
        self.mask = np.zeros((cap, 3), np.uint8)
        self.count = self.t = self.draws = 0
        self.n_greedy = 0

    def _step(self, a):
        r = self.env.step(np.array([a], np.uint8))
        k = self.count % self.cap
        self.frames[k], self.act[k], self.rew[k] = r["frames"][0], a, r["reward"][0]
        self.done[k], self.mask[k] = r["done"][0], r["mask"][0]
        self.count += 1
        self.t += 1
        return bool(r["done"][0]), np.float32(r["reward"][0])

    def episode(self):
        """play_episode (utils.jl:198-259) with store! of every transition."""
        L, ep = 0, np.float32(0)
        while True:
            a = explore(self.seed, 0, self.t, self.eps)
            if a is None:
                x = self.env.states().astype(np.float32)
                a = first_argmax(oracle.qnet_forward(self.bs, self.C, self.th, x)[0])
                self.n_greedy += 1
            done, r = self._step(a)
            ep = np.float32(ep + r)
            L += 1
            if done:
                return L, ep

    def fill(self):
        played = 0
        while played <= self.cap:
            played += self.episode()[0]
        return played

    def step(self, nb):
        """One episode, one B-sample update, update_target_net! at nb % rate == 0,
        epsilon decay. Returns (episode reward, loss)."""
        _, ep = self.episode()
        ids = floyd(self.seed, self.draws, min(self.count, self.cap), self.B)
        self.draws += 1
        f = self.frames[ids]
        C = self.C
        loss, g, _ = oracle.dqn_loss_grad(self.bs, C, self.th, self.tt, f[:, :C], self.act[ids], self.rew[ids],
                                          f[:, 1:], self.done[ids], self.mask[ids], self.gamma)
        self.last_grad, self.last_ids = g, ids
        self.th, self.acc = oracle.rmsprop(self.th, self.acc, g.astype(np.float32))
        if nb % self.rate == 0:
            self.tt = self.th.copy()
        self.eps = max(np.float32(self.eps - np.float32(self.decay)), np.float32(self.eps_end))
        return ep, loss
