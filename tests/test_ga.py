"""GA semantics vs the reference (pathnet.py:32-87, doom_pathnet.py:211-293)."""
import numpy as np
import pytest

from pathnet_gym_amd.algo.ga import (Population, compact_active, decode_path, express, get_geopath, mutation,
                                     mutation_down, select_two_candi)
from pathnet_gym_amd.config import FITNESS_PENDING


def test_get_geopath_exactly_n_per_layer():
    rng = np.random.RandomState(0)
    for _ in range(50):
        g = get_geopath(4, 10, 4, rng)
        assert g.shape == (4, 10)
        assert set(np.unique(g)) <= {0.0, 1.0}
        assert (g.sum(1) == 4).all()


def test_mutation_probabilities_match_reference_formula():
    """active module moves with p=2/(L*N); inactive module activates one with p=2/(L*(M-N)*M)."""
    L, M, N = 4, 10, 4
    rng = np.random.RandomState(1)
    trials = 4000
    moved = 0
    act_events = 0
    n_active = n_inactive = 0
    for _ in range(trials):
        g = np.zeros((L, M), np.float32)
        g[:, :N] = 1
        # replicate the reference loop with an instrumented copy of the RNG stream
        r2 = np.random.RandomState(rng.randint(1 << 30))
        for i in range(L):
            for j in range(M):
                if g[i, j] == 1:
                    n_active += 1
                    if int(r2.rand() * L * N) <= 1:
                        moved += 1
                        g[i, j] = 0
                        g[i, r2.randint(0, M)] = 1
                else:
                    n_inactive += 1
                    if int(r2.rand() * L * (M - N) * M) <= 1:
                        act_events += 1
                        g[i, r2.randint(0, M)] = 1
    p_move = moved / n_active
    p_act = act_events / n_inactive
    assert abs(p_move - 2 / (L * N)) < 0.015
    assert abs(p_act - 2 / (L * (M - N) * M)) < 0.004


def test_mutation_same_stream_as_reference_loop():
    """mutation() consumes the RNG exactly like the reference loop (same results for same seed)."""
    L, M, N = 3, 6, 2
    g0 = get_geopath(L, M, N, np.random.RandomState(3))
    a = mutation(g0.copy(), L, M, N, np.random.RandomState(9))
    r = np.random.RandomState(9)
    b = g0.copy()
    for i in range(L):
        for j in range(M):
            if b[i, j] == 1:
                if int(r.rand() * L * N) <= 1:
                    b[i, j] = 0
                    b[i, r.randint(0, M)] = 1
            else:
                if int(r.rand() * L * (M - N) * M) <= 1:
                    b[i, r.randint(0, M)] = 1
    assert np.array_equal(a, b)


def test_mutation_down_moves_to_lower_indices_clamped():
    rng = np.random.RandomState(0)
    L, M, N = 1, 10, 1
    for _ in range(200):
        g = np.zeros((L, M), np.float32)
        g[0, 2] = 1
        out = mutation_down(g, L, M, 1, rng)
        idx = np.nonzero(out[0])[0]
        assert len(idx) == 1 and idx[0] <= 2    # offset in {-4..-1} clamped at 0, or unchanged


def test_select_two_candi_distinct():
    rng = np.random.RandomState(0)
    for _ in range(100):
        a, b = select_two_candi(5, rng)
        assert a != b and 0 <= a < 5 and 0 <= b < 5


def test_decode_and_express():
    g = np.zeros((2, 4), np.float32)
    g[0, [1, 3]] = 1
    fr = np.zeros((2, 4), np.float32)
    fr[1, 0] = 1
    e = express(g, fr)
    assert e[1, 0] == 1 and e[0, 1] == 1 and e.sum() == 3
    d = decode_path(g)
    assert list(d[0]) == [1, 3] and list(d[1]) == []
    idx, cnt = compact_active(e[None])
    assert list(cnt[0]) == [2, 1] and list(idx[0, 0, :2]) == [1, 3] and idx[0, 0, 2] == -1


def test_tournament_semantics():
    pop = Population(P=6, L=3, M=5, N=2, B=3, seed=4)
    cand = list(pop.candidates[0])
    assert len(cand) == 3 and len(set(cand)) == 3
    fit = np.full(6, FITNESS_PENDING, np.float32)
    # not all candidates have a fitness yet -> nothing happens
    fit[cand[0]] = 5.0
    fit[cand[1]] = 1.0
    assert pop.step(fit) == []
    fit[cand[2]] = 3.0
    winner_g = pop.genotypes[cand[0]].copy()
    ev = pop.step(fit.copy())
    assert len(ev) == 1 and ev[0].winner == cand[0] and ev[0].winner_fitness == 5.0
    # winner unchanged, all B scores reset (doom_pathnet.py:267)
    assert np.array_equal(pop.genotypes[cand[0]], winner_g)
    assert all(pop.fitness[c] == FITNESS_PENDING for c in cand)
    assert pop.generation == 1
    # a new candidate set was drawn
    assert len(pop.candidates) == 1


def test_losers_are_mutated_copies_of_winner():
    pop = Population(P=3, L=4, M=10, N=4, B=3, seed=11)
    cand = pop.candidates[0]
    fit = np.array([0.0, 0.0, 0.0], np.float32)
    fit[cand[1]] = 9.0
    w = cand[1]
    gw = pop.genotypes[w].copy()
    pop.step(fit)
    for c in cand:
        if c != w:
            diff = np.abs(pop.genotypes[c] - gw).sum()
            assert diff <= 8    # only a few mutation events away from the winner


def test_freeze_union_vs_reference():
    pop = Population(P=4, L=2, M=4, N=1, B=2, seed=0)
    pop.genotypes[0] = np.array([[1, 0, 0, 0], [0, 1, 0, 0]], np.float32)
    pop.genotypes[1] = np.array([[0, 0, 1, 0], [0, 0, 0, 1]], np.float32)
    f1 = pop.freeze(0, union=True)
    f2 = pop.freeze(1, union=True)
    assert f2.sum() == 4 and f1.sum() == 2
    pop.frozen[:] = 0
    pop.freeze(0, union=False)
    f3 = pop.freeze(1, union=False)      # reference quirk: replaces (game_ac_network.py:490-491)
    assert f3.sum() == 2 and f3[0, 2] == 1


def test_concurrent_tournaments_disjoint():
    pop = Population(P=12, L=2, M=4, N=2, B=3, seed=0, concurrent=4)
    flat = [i for c in pop.candidates for i in c]
    assert len(pop.candidates) == 4 and len(set(flat)) == 12


def test_state_dict_roundtrip_keeps_rng_stream():
    a = Population(P=5, L=3, M=4, N=2, B=2, seed=7)
    sd = a.state_dict()
    b = Population(P=5, L=3, M=4, N=2, B=2, seed=99)
    b.load_state_dict(sd)
    fit = np.arange(5, dtype=np.float32)
    a.step(fit.copy())
    b.step(fit.copy())
    assert np.array_equal(a.genotypes, b.genotypes)
    assert a.candidates == b.candidates


# ---------------------------------------------------------------------------
# counter-based (device) GA mirror
# ---------------------------------------------------------------------------
def _drive(pop, steps, seed):
    rng = np.random.RandomState(seed)
    evs = []
    for t in range(steps):
        f = pop.fitness.copy()
        fresh = rng.rand(pop.P) < 0.4
        f[fresh] = rng.randint(-21, 22, int(fresh.sum())).astype(np.float32)
        evs += pop.step(f, t)
    return evs


def test_counter_ga_deterministic_and_disjoint():
    from pathnet_gym_amd.algo.ga_device import CounterPopulation
    a = CounterPopulation(24, 5, 10, 4, 3, seed=7, concurrent=4)
    b = CounterPopulation(24, 5, 10, 4, 3, seed=7, concurrent=4)
    ea, eb = _drive(a, 60, 1), _drive(b, 60, 1)
    assert len(ea) > 20 and [e.winner for e in ea] == [e.winner for e in eb]
    assert np.array_equal(a.genotypes, b.genotypes) and np.array_equal(a.slots, b.slots)
    used = a.slots[a.slots >= 0]
    assert len(set(used.tolist())) == len(used)                     # disjoint tournaments
    for e in ea:
        assert e.winner == e.candidates[int(np.argmax(e.scores))]
    c = CounterPopulation(24, 5, 10, 4, 3, seed=8, concurrent=4)
    _drive(c, 60, 1)
    assert not np.array_equal(a.genotypes, c.genotypes)


def test_counter_mutation_rates_match_reference_operator():
    from pathnet_gym_amd.algo.ga_device import counter_mutation
    L, M, N = 4, 10, 4
    moved = trials_a = 0
    for gen in range(3000):
        g = np.zeros((L, M), np.float32)
        g[:, :N] = 1
        before = g.copy()
        counter_mutation(g, L, M, N, seed=123, gen=gen, path=5)
        trials_a += 1
        moved += before[0, 0] == 1 and g[0, 0] == 0
    # P[int(U*L*N) <= 1] = 2/(L*N), times P[the random target is not module 0 itself] = (M-1)/M
    assert abs(moved / trials_a - 2 / (L * N) * (M - 1) / M) < 0.02


def test_counter_mutation_vectorised_draws_match_scalar():
    """algo/ga_device.counter_mutation draws its 2 L M counter-hash numbers in one numpy pass; the decisions equal
    the scalar walk's (the device GA kernel's oracle) on random genotypes, seeds, generations and paths."""
    from pathnet_gym_amd.algo.ga_device import counter_mutation, counter_mutation_scalar
    rng = np.random.RandomState(0)
    for _ in range(500):
        L, M = int(rng.randint(1, 6)), int(rng.randint(2, 11))
        N = int(rng.randint(1, M))
        g = (rng.rand(L, M) < 0.5).astype(np.float32)
        seed, gen, path = int(rng.randint(0, 2 ** 32 - 1)), int(rng.randint(0, 10 ** 7)), int(rng.randint(0, 4096))
        assert np.array_equal(counter_mutation(g.copy(), L, M, N, seed, gen, path),
                              counter_mutation_scalar(g.copy(), L, M, N, seed, gen, path))
