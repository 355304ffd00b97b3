"""Restatement of the device's counter-based RNG draws (test infrastructure).

The reference draws actions (utils.jl:161-166) and replay samples
(utils.jl:280-287) from Julia's unseeded global RNG, so no run of it is
reproducible; the device replaces that stream with counter-based draws
(snk_common.hpp rng_hash). These helpers restate those draws in Python so the
parity tests can replay a device run on the CPU oracle decision by decision.
"""
import numpy as np

M64 = (1 << 64) - 1


def splitmix64(x: int) -> int:
    z = (x + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def rng_hash(seed: int, a: int, b: int) -> int:
    return splitmix64(splitmix64(seed ^ ((a * 0xD1B54A32D192ED03) & M64)) ^ b)


def rng_uniform(h: int) -> np.float32:
    return np.float32(h >> 40) * np.float32(1.0 / 16777216.0)


def explore(seed: int, env: int, t: int, epsilon) -> int | None:
    """epsilon_greedy's coin (utils.jl:161): the random action index when
    Float32(rand()) < epsilon, else None (take the greedy action)."""
    if rng_uniform(rng_hash(seed, env, t)) < np.float32(epsilon):
        return (rng_hash(seed ^ 0xA5A5A5A5A5A5A5A5, env, t) >> 32) % 3
    return None


def first_argmax(q) -> int:
    """av[argmax(Q)] with Julia's first-maximum tie rule (utils.jl:167)."""
    a = 0
    if q[1] > q[a]:
        a = 1
    if q[2] > q[a]:
        a = 2
    return a


def floyd(seed: int, draw: int, n_len: int, batch: int) -> list[int]:
    """sample(rpb) without replacement (utils.jl:280-287) as the device draws
    it: Floyd's algorithm over rng_hash(seed, draw, n)."""
    B = min(batch, n_len)
    chosen, out = set(), []
    for n in range(B):
        t = (rng_hash(seed, draw, n) * (n_len - B + n + 1)) >> 64
        v = n_len - B + n if t in chosen else t
        chosen.add(v)
        out.append(v)
    return out


TRAINER_SAMPLE_SALT = 0x5A4D504C45   # snk_trainer.hip: replay draws use cfg.seed ^ this


def _splitmix64_np(x):
    z = x + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def rng_hash_np(seed: int, a: np.ndarray, b: int) -> np.ndarray:
    """rng_hash over an array of first counters (uint64 wrap-around arithmetic)."""
    with np.errstate(over="ignore"):
        a = np.asarray(a, np.uint64)
        return _splitmix64_np(_splitmix64_np(np.uint64(seed) ^ (a * np.uint64(0xD1B54A32D192ED03))) ^ np.uint64(b))


def explore_np(seed: int, n_envs: int, t: int, epsilon) -> np.ndarray:
    """explore() for envs 0..n_envs-1 at step t: the random action index, or -1
    where epsilon_greedy takes the greedy action."""
    e = np.arange(n_envs, dtype=np.uint64)
    u = (rng_hash_np(seed, e, t) >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    r = ((rng_hash_np(seed ^ 0xA5A5A5A5A5A5A5A5, e, t) >> np.uint64(32)) % np.uint64(3)).astype(np.int64)
    return np.where(u < np.float32(epsilon), r, -1)


def first_argmax_np(q: np.ndarray) -> np.ndarray:
    """first_argmax over rows of q [n, 3]."""
    a = np.zeros(len(q), np.int64)
    a = np.where(q[:, 1] > q[np.arange(len(q)), a], 1, a)
    a = np.where(q[:, 2] > q[np.arange(len(q)), a], 2, a)
    return a
