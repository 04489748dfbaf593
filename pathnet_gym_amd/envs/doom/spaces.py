"""Action-space types and adapters (reference ``wrappers/multi_discrete.py``).

``DiscreteToMultiDiscrete(md, options)`` turns a MultiDiscrete space into a
Discrete one:
  * options None  -> n = 1 + dims; action i>0 presses dim i-1 at its max
  * options list  -> n = 1 + len(list); action i>0 presses dim list[i-1]
  * options dict  -> n = len(dict); keys must be 0..n-1 in order, every value
                     must be inside the MultiDiscrete space
``BoxToMultiDiscrete(md, options)`` rounds a continuous vector onto the
selected dims (all dims when options is None).
"""
from __future__ import annotations

import numpy as np


class SpaceError(ValueError):
    pass


class Discrete:
    def __init__(self, n: int):
        self.n = int(n)

    def sample(self, rng=np.random):
        return int(rng.randint(self.n))

    def contains(self, x) -> bool:
        return 0 <= int(x) < self.n


class Box:
    def __init__(self, low, high, shape=None, dtype=np.float32):
        self.low = np.asarray(low)
        self.high = np.asarray(high)
        self.shape = tuple(shape) if shape is not None else self.low.shape
        self.dtype = dtype

    def sample(self, rng=np.random):
        return rng.uniform(self.low, self.high, size=self.shape)

    def contains(self, x) -> bool:
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))


class MultiDiscrete:
    """[[low, high], ...] per dimension (old gym API)."""

    def __init__(self, ranges):
        r = np.asarray(ranges)
        self.low = r[:, 0]
        self.high = r[:, 1]
        self.num_discrete_space = len(r)

    def sample(self, rng=np.random):
        return [int(rng.randint(lo, hi + 1)) for lo, hi in zip(self.low, self.high)]

    def contains(self, x) -> bool:
        x = np.asarray(x)
        return x.shape == (self.num_discrete_space,) and bool(np.all(x >= self.low) and np.all(x <= self.high))


class DiscreteToMultiDiscrete(Discrete):
    def __init__(self, multi_discrete: MultiDiscrete, options=None):
        if not isinstance(multi_discrete, MultiDiscrete):
            raise SpaceError("DiscreteToMultiDiscrete needs a MultiDiscrete space")
        self.multi_discrete = multi_discrete
        d = multi_discrete.num_discrete_space
        self.num_discrete_space = d
        if options is None:
            options = list(range(d))
        if isinstance(options, list):
            if len(options) > d:
                raise SpaceError("more options than dimensions")
            self.n = len(options) + 1
            self.mapping = {i: [0] * d for i in range(self.n)}
            for i, dim in enumerate(options):
                if not 0 <= dim < d:
                    raise SpaceError(f"dimension {dim} out of range")
                self.mapping[i + 1][dim] = int(multi_discrete.high[dim])
        elif isinstance(options, dict):
            self.n = len(options)
            for i, key in enumerate(options):
                if i != key:
                    raise SpaceError(f"DiscreteToMultiDiscrete must contain ordered keys; item {i} has key {key}")
                if not multi_discrete.contains(options[key]):
                    raise SpaceError(f"mapping for key {key} is not inside the MultiDiscrete space: {options[key]}")
            self.mapping = {k: list(v) for k, v in options.items()}
        else:
            raise SpaceError("DiscreteToMultiDiscrete - invalid options")

    def __call__(self, discrete_action):
        return self.mapping[int(discrete_action)]


class BoxToMultiDiscrete(Box):
    def __init__(self, multi_discrete: MultiDiscrete, options=None):
        if not isinstance(multi_discrete, MultiDiscrete):
            raise SpaceError("BoxToMultiDiscrete needs a MultiDiscrete space")
        self.multi_discrete = multi_discrete
        d = multi_discrete.num_discrete_space
        self.num_discrete_space = d
        if options is None:
            options = list(range(d))
        if not isinstance(options, list):
            raise SpaceError("BoxToMultiDiscrete - invalid options")
        if len(options) > d:
            raise SpaceError("more options than dimensions")
        super().__init__([multi_discrete.low[x] for x in options], [multi_discrete.high[x] for x in options])
        self.mapping = {i: dim for i, dim in enumerate(options)}

    def __call__(self, box_action):
        out = [0] * self.num_discrete_space
        for i, dim in self.mapping.items():
            out[dim] = int(round(float(box_action[i]), 0))
        return out
