"""PathNet genetic algorithm: genotypes, mutation, B-way tournament.

Exact semantics of the reference (``pathnet.py:32-87``, ``doom_pathnet.py:211-293``):

* genotype = L x M array of {0,1}; initial genotypes have exactly N active
  modules per layer (``get_geopath``, rejection sampling).
* ``mutation``: each active module moves to a uniformly random module of the
  same layer with prob 2/(L*N) (``int(U*L*N) <= 1``); each inactive module
  activates a random module with prob 2/(L*(M-N)*M).  The active count can
  therefore shrink or grow.
* tournament: sample B distinct candidates; once all have a fitness
  (!= -1000) the argmax wins, every loser becomes ``mutation(copy(winner))``,
  ALL B fitness values reset to -1000, a new B is drawn.
* expressed mask = genotype OR frozen path.

The whole GA state (genotype table, fitness vector, candidate sets, RNG) is
replicated on every rank; all ranks feed identical fitness vectors (from the
fused all-reduce, see ``parallel/comm.py``) into an identically seeded
``numpy.random.RandomState`` and so take identical decisions without a
coordinator process.  This replaces the reference's dedicated coordinator
worker (``doom_pathnet.py:202``) polling PS scalars.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from ..config import FITNESS_PENDING


# ---------------------------------------------------------------------------
# single-genotype operators (numpy, canonical float [L,M] or uint8)
# ---------------------------------------------------------------------------
def get_geopath(L: int, M: int, N: int, rng: np.random.RandomState) -> np.ndarray:
    """Random genotype with exactly N distinct active modules per layer (pathnet.py:78-87)."""
    if N > M:
        raise ValueError("N must be <= M")
    g = np.zeros((L, M), dtype=np.float32)
    for i in range(L):
        j = 0
        while j < N:
            r = int(rng.rand() * M)
            if g[i, r] == 0.0:
                g[i, r] = 1.0
                j += 1
    return g


def mutation(g: np.ndarray, L: int, M: int, N: int, rng: np.random.RandomState) -> np.ndarray:
    """Reference mutation operator, in place + returned (pathnet.py:50-63)."""
    for i in range(L):
        for j in range(M):
            if g[i, j] == 1:
                if int(rng.rand() * L * N) <= 1:
                    g[i, j] = 0
                    g[i, rng.randint(0, M)] = 1
            else:
                if int(rng.rand() * L * (M - N) * M) <= 1:
                    g[i, rng.randint(0, M)] = 1
    return g


def mutation_down(g: np.ndarray, L: int, M: int, N: int, rng: np.random.RandomState) -> np.ndarray:
    """Local-shift mutation (pathnet.py:32-48): move by an offset in {-4..-1}, clamped."""
    for i in range(L):
        for j in range(M):
            if g[i, j] == 1:
                if int(rng.rand() * L * N) <= 1:
                    g[i, j] = 0
                    off = rng.randint(-2, 2) - 2
                    t = min(max(j + off, 0), M - 1)
                    g[i, t] = 1
    return g


def select_two_candi(M: int, rng: np.random.RandomState):
    """Two distinct indices in [0,M) (pathnet.py:65-76)."""
    a = int(rng.rand() * M)
    while True:
        b = int(rng.rand() * M)
        if b != a:
            return a, b


def decode_path(g: np.ndarray) -> List[np.ndarray]:
    """Active module indices per layer (doom_pathnet.py:241 decodePath)."""
    return [np.where(row == 1.0)[0] for row in np.asarray(g, dtype=np.float32)]


def express(g: np.ndarray, frozen: np.ndarray) -> np.ndarray:
    """Expressed mask = genotype OR frozen path (doom_pathnet.py:216-221,261-266)."""
    return ((np.asarray(g) > 0.5) | (np.asarray(frozen) > 0.5)).astype(np.float32)


# ---------------------------------------------------------------------------
# population / tournament state
# ---------------------------------------------------------------------------
@dataclass
class TournamentEvent:
    generation: int
    step: int
    candidates: List[int]
    winner: int
    winner_fitness: float
    scores: List[float]


@dataclass
class Population:
    """Replicated GA state for the whole population (all ranks)."""
    P: int
    L: int
    M: int
    N: int
    B: int = 3
    seed: int = 1
    mutation_kind: str = "ref"
    concurrent: int = 1
    genotypes: np.ndarray = field(init=False)        # [P, L, M] float32 {0,1}, evolvable part
    frozen: np.ndarray = field(init=False)           # [L, M] float32 union of frozen paths
    fitness: np.ndarray = field(init=False)          # [P] float32 (-1000 pending)
    candidates: List[List[int]] = field(init=False)  # active tournaments
    generation: int = field(init=False, default=0)
    history: List[TournamentEvent] = field(init=False, default_factory=list)

    def __post_init__(self):
        if self.B > self.P:
            raise ValueError(f"tournament size B={self.B} > population {self.P}")
        self.rng = np.random.RandomState(self.seed)
        self.frozen = np.zeros((self.L, self.M), np.float32)
        self.fitness = np.full(self.P, FITNESS_PENDING, np.float32)
        self.init_genotypes()

    # -- task boundaries ------------------------------------------------------
    def init_genotypes(self):
        """Fresh random genotypes (doom_pathnet.py:213-221) + fresh tournaments."""
        self.genotypes = np.stack([get_geopath(self.L, self.M, self.N, self.rng)
                                   for _ in range(self.P)])
        self.fitness[:] = FITNESS_PENDING
        self.candidates = []
        self._draw_candidates()

    def _draw_candidates(self):
        """Draw disjoint candidate sets (doom_pathnet.py:227-229,268-270)."""
        busy = set(i for c in self.candidates for i in c)
        while len(self.candidates) < self.concurrent:
            pool = np.array([i for i in range(self.P) if i not in busy], dtype=np.int64)
            if len(pool) < self.B:
                break
            perm = pool.copy()
            self.rng.shuffle(perm)
            c = [int(x) for x in perm[: self.B]]
            self.candidates.append(c)
            busy.update(c)

    def expressed(self) -> np.ndarray:
        """[P, L, M] expressed masks."""
        return ((self.genotypes > 0.5) | (self.frozen[None] > 0.5)).astype(np.float32)

    # -- tournament -------------------------------------------------------------
    def mutate(self, g):
        if self.mutation_kind == "down":
            return mutation_down(g, self.L, self.M, self.N, self.rng)
        return mutation(g, self.L, self.M, self.N, self.rng)

    def step(self, fitness: np.ndarray, global_step: int = 0) -> List[TournamentEvent]:
        """Feed the latest fitness vector; run every ready tournament.

        Returns the list of tournaments that fired (possibly empty).  The
        genotype table is updated in place; callers push ``expressed()`` to
        the device afterwards.
        """
        self.fitness[:] = fitness
        events = []
        remaining = []
        for cand in self.candidates:
            scores = self.fitness[cand]
            if np.any(scores == FITNESS_PENDING):
                remaining.append(cand)
                continue
            w = cand[int(np.argmax(scores))]
            ev = TournamentEvent(self.generation, global_step, list(cand), w,
                                 float(self.fitness[w]), [float(s) for s in scores])
            for i in cand:
                if i != w:
                    self.genotypes[i] = self.mutate(self.genotypes[w].copy())
                self.fitness[i] = FITNESS_PENDING
            self.generation += 1
            self.history.append(ev)
            events.append(ev)
        self.candidates = remaining
        if events:
            self._draw_candidates()
        return events

    def best(self) -> int:
        """Index of the path to freeze at task end (last tournament winner, ref :274)."""
        if self.history:
            return self.history[-1].winner
        return 0

    def freeze(self, idx: int, union: bool = True) -> np.ndarray:
        """Freeze path ``idx``; returns the new frozen mask (doom_pathnet.py:274-283)."""
        g = self.genotypes[idx] > 0.5
        if union:
            self.frozen = ((self.frozen > 0.5) | g).astype(np.float32)
        else:
            self.frozen = g.astype(np.float32)
        return self.frozen.copy()

    # -- (de)serialisation ------------------------------------------------------
    def state_dict(self):
        st = self.rng.get_state()
        return {
            "genotypes": self.genotypes.astype(np.uint8),
            "frozen": self.frozen.astype(np.uint8),
            "fitness": self.fitness.copy(),
            "candidates": np.array(self.candidates, dtype=np.int64).reshape(-1, self.B) if self.candidates
            else np.zeros((0, self.B), np.int64),
            "generation": np.array(self.generation, dtype=np.int64),
            "rng_keys": st[1].astype(np.uint32),
            "rng_pos": np.array([st[2], st[3]], dtype=np.int64),
            "rng_gauss": np.array([st[4]], dtype=np.float64),
        }

    def load_state_dict(self, d):
        self.genotypes = np.asarray(d["genotypes"]).astype(np.float32)
        self.frozen = np.asarray(d["frozen"]).astype(np.float32)
        self.fitness = np.asarray(d["fitness"]).astype(np.float32).copy()
        self.candidates = [list(map(int, c)) for c in np.asarray(d["candidates"])]
        self.generation = int(np.asarray(d["generation"]).reshape(-1)[0])
        pos = np.asarray(d["rng_pos"])
        self.rng.set_state(("MT19937", np.asarray(d["rng_keys"]).astype(np.uint32), int(pos[0]), int(pos[1]),
                            float(np.asarray(d["rng_gauss"])[0])))


def compact_active(expressed: np.ndarray):
    """[P,L,M] mask -> (act_idx [P,L,M] int32 padded with -1, act_cnt [P,L] int32).

    The compacted index list is what the HIP grouped-GEMM kernels consume:
    each (path, layer) has up to M active modules; count 0 is legal (an empty
    layer outputs zeros, the reference's mask semantics).
    """
    P, L, M = expressed.shape
    idx = np.full((P, L, M), -1, np.int32)
    cnt = np.zeros((P, L), np.int32)
    for p in range(P):
        for l in range(L):
            a = np.nonzero(expressed[p, l] > 0.5)[0]
            idx[p, l, : len(a)] = a
            cnt[p, l] = len(a)
    return idx, cnt
