"""Counter-based tournament GA that runs ON DEVICE (csrc/ga.hip), with a bit-exact numpy mirror.

The reference GA (``pathnet.py:50-87``, ``doom_pathnet.py:225-270``) draws
from numpy's global MT19937 stream; ``algo/ga.py:Population`` reproduces that
exactly on the host.  This variant keeps the SAME operators -- B-way
tournament on the latest fitness, losers := mutated copy of the winner, all
candidates reset to pending, disjoint redraw -- and the same mutation
probabilities (active module moves with P[int(U*L*N) <= 1], an inactive one
activates a random module with P[int(U*L*(M-N)*M) <= 1]), but every random
number is a pure function of (seed, generation, path, layer, draw): a Wang
hash chain.  That makes the whole GA step a data-parallel kernel that can live
in the optimizer hipGraph right after the fitness all-reduce (SURVEY.md
section 2.8 K17/K18, section 7.1 "GA kernels"), with no host round trip, and
replicated ranks stay identical by construction.

Tournaments live in C fixed slots (``slots [C, B]``, -1 = empty).  The host
mirror (``CounterPopulation``) and the device kernel take identical decisions,
which the GPU tests check generation by generation.
"""
from __future__ import annotations

from typing import List

import numpy as np

from ..config import FITNESS_PENDING
from .ga import Population, TournamentEvent

M32 = 0xFFFFFFFF
DRAW_KEY = 0xFFFF           # x-coordinate of candidate-draw random numbers
MAX_ATTEMPTS = 64           # rejection-sampling attempts per candidate before the ascending scan


def wang(x: int) -> int:
    x &= M32
    x = (x ^ 61) ^ (x >> 16)
    x = (x * 9) & M32
    x ^= x >> 4
    x = (x * 0x27D4EB2D) & M32
    x ^= x >> 15
    return x


def ga_rand(seed: int, gen: int, x: int, y: int, z: int) -> int:
    h = wang(wang(seed) ^ (gen & M32))
    h = wang(h ^ (x & M32))
    return wang(h ^ (((y & 0xFFFF) << 16) + (z & 0xFFFF)))


def wang_np(x: np.ndarray) -> np.ndarray:
    """``wang`` on a uint64 array holding 32-bit values (element-wise, bit-identical)."""
    x = x & M32
    x = (x ^ 61) ^ (x >> 16)
    x = (x * 9) & M32
    x ^= x >> 4
    x = (x * 0x27D4EB2D) & M32
    x ^= x >> 15
    return x


def ga_rand_np(seed: int, gen: int, x: int, y: np.ndarray, z: np.ndarray) -> np.ndarray:
    """``ga_rand`` over arrays of (y, z) draws (uint64 in, uint64 out)."""
    h = wang(wang(seed) ^ (gen & M32))
    h = wang(h ^ (x & M32))
    return wang_np(np.uint64(h) ^ (((y & 0xFFFF) << 16) + (z & 0xFFFF)))


def counter_mutation(g: np.ndarray, L: int, M: int, N: int, seed: int, gen: int, path: int) -> np.ndarray:
    """Reference mutation operator with counter-based draws (in place, returned).  The 2 L M draws are independent of
    the genotype, so they are computed in one vectorised pass; the per-layer walk over the modules stays sequential
    (a move can activate a module that a later step of the same layer reads)."""
    ka = L * N
    ki = L * (M - N) * M
    ll, mm = np.meshgrid(np.arange(L, dtype=np.uint64), np.arange(M, dtype=np.uint64), indexing="ij")
    h0 = ga_rand_np(seed, gen, path, ll, 2 * mm).tolist()
    h1 = ga_rand_np(seed, gen, path, ll, 2 * mm + 1).tolist()
    for l in range(L):
        row0, row1 = h0[l], h1[l]
        for m in range(M):
            u24 = row0[m] >> 8                # U = u24 / 2^24;  int(U*K) <= 1  <=>  u24*K < 2^25
            if g[l, m] == 1:
                if u24 * ka < (1 << 25):
                    g[l, m] = 0
                    g[l, row1[m] % M] = 1
            elif u24 * ki < (1 << 25):
                g[l, row1[m] % M] = 1
    return g


def counter_mutation_scalar(g: np.ndarray, L: int, M: int, N: int, seed: int, gen: int, path: int) -> np.ndarray:
    """The scalar form of counter_mutation (the oracle its vectorised draws are tested against)."""
    ka = L * N
    ki = L * (M - N) * M
    for l in range(L):
        for m in range(M):
            h0 = ga_rand(seed, gen, path, l, 2 * m)
            h1 = ga_rand(seed, gen, path, l, 2 * m + 1)
            u24 = h0 >> 8
            if g[l, m] == 1:
                if u24 * ka < (1 << 25):
                    g[l, m] = 0
                    g[l, h1 % M] = 1
            elif u24 * ki < (1 << 25):
                g[l, h1 % M] = 1
    return g


def draw_slot(seed: int, key_gen: int, slot: int, P: int, B: int, busy: np.ndarray) -> List[int]:
    """B distinct non-busy path indices (marks them busy); [] if fewer than B are free."""
    if int((~busy).sum()) < B:
        return []
    out = []
    attempt = 0
    while len(out) < B and attempt < MAX_ATTEMPTS * B:
        i = ga_rand(seed, key_gen, DRAW_KEY, slot, attempt) % P
        attempt += 1
        if not busy[i]:
            busy[i] = True
            out.append(int(i))
    i = 0
    while len(out) < B:                      # deterministic fallback: ascending scan
        if not busy[i]:
            busy[i] = True
            out.append(i)
        i += 1
    return out


class CounterPopulation(Population):
    """Population whose tournaments/mutations are the counter-based device GA (host mirror)."""

    def __post_init__(self):
        self.seed32 = (self.seed * 2654435761) & M32
        self.draw_round = 0
        super().__post_init__()

    def init_genotypes(self):
        """Fresh genotypes (host MT19937, as the reference) and a fresh fill of the C tournament slots."""
        self.slots = np.full((self.concurrent, self.B), -1, np.int64)
        super().init_genotypes()

    def _draw_candidates(self):
        """Fill empty slots at task start (host side; the slot table is uploaded to the device)."""
        busy = np.zeros(self.P, bool)
        for c in range(self.concurrent):
            if self.slots[c, 0] >= 0:
                busy[self.slots[c]] = True
        key = 0x80000000 | (self.draw_round & 0x7FFFFFFF)
        self.draw_round += 1
        for c in range(self.concurrent):
            if self.slots[c, 0] < 0:
                got = draw_slot(self.seed32, key, c, self.P, self.B, busy)
                if got:
                    self.slots[c] = got
        self.candidates = [list(map(int, r)) for r in self.slots if r[0] >= 0]

    def step(self, fitness: np.ndarray, global_step: int = 0) -> List[TournamentEvent]:
        self.fitness[:] = fitness
        C = self.concurrent
        ready = np.zeros(C, bool)
        winners = np.full(C, -1, np.int64)
        for c in range(C):
            cand = self.slots[c]
            if cand[0] < 0:
                continue
            sc = self.fitness[cand]
            if np.any(sc == FITNESS_PENDING):
                continue
            ready[c] = True
            winners[c] = cand[int(np.argmax(sc))]
        events = []
        gen_of = np.full(C, -1, np.int64)
        for c in range(C):
            if not ready[c]:
                continue
            gen = self.generation
            gen_of[c] = gen
            cand = self.slots[c]
            w = int(winners[c])
            ev = TournamentEvent(gen, global_step, [int(x) for x in cand], w, float(self.fitness[w]),
                                 [float(self.fitness[i]) for i in cand])
            for i in cand:
                if i != w:
                    g = self.genotypes[w].copy()
                    self.genotypes[i] = counter_mutation(g, self.L, self.M, self.N, self.seed32, gen, int(i))
            self.generation += 1
            self.history.append(ev)
            events.append(ev)
        for c in range(C):
            if ready[c]:
                self.fitness[self.slots[c]] = FITNESS_PENDING
        if events:
            busy = np.zeros(self.P, bool)
            for c in range(C):
                if not ready[c] and self.slots[c, 0] >= 0:
                    busy[self.slots[c]] = True
            for c in range(C):
                if ready[c]:
                    got = draw_slot(self.seed32, int(gen_of[c]), c, self.P, self.B, busy)
                    self.slots[c] = got if got else -1
            self.candidates = [list(map(int, r)) for r in self.slots if r[0] >= 0]
        return events

    def state_dict(self):
        d = super().state_dict()
        d["slots"] = self.slots.astype(np.int64)
        d["draw_round"] = np.array(self.draw_round, dtype=np.int64)
        return d

    def load_state_dict(self, d):
        super().load_state_dict(d)
        if "slots" in d:
            self.slots = np.asarray(d["slots"]).astype(np.int64)
            self.draw_round = int(np.asarray(d["draw_round"]).reshape(-1)[0])
            self.candidates = [list(map(int, r)) for r in self.slots if r[0] >= 0]
