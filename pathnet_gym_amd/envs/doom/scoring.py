"""MetaDoom 9-level curriculum scoring (reference ``doom_env.py:288-454``).

Engine-independent logic of ``MetaDoomEnv``:

* standardised episode score in [0, 1000]: with min/target from the level
  table and max = min + (target - min)/0.99 (target = 99th percentile),
  ``round(1000*(r - min)/(max - min), 4)`` clipped to [0, 1000];
* per level, the last ``min_tries_for_avg`` scores are kept (a new episode
  inserts 0 at the front); the level average is over at most
  ``average_over`` entries;
* a level unlocks the next one when its average >= ``passing_grade``
  (checked from the second-to-last level downwards);
* the next level is the unlocked level with the LOWEST average (ties: the
  first), level 0 by default;
* total reward = sum of level averages + 50*levels if every level's average
  >= 990; step reward = change of the total (the first step of an episode
  returns the whole total, as in the reference's quirk).
"""
from __future__ import annotations

from typing import List

from .constants import DOOM_SETTINGS, MIN_SCORE, NUM_LEVELS, TARGET_SCORE


class MetaDoomScorer:
    def __init__(self, average_over: int = 10, passing_grade: float = 600, min_tries_for_avg: int = 5):
        self.average_over = average_over
        self.passing_grade = passing_grade
        self.min_tries_for_avg = min_tries_for_avg
        self.scores: List[List[float]] = [[] for _ in range(NUM_LEVELS)]
        self.locked_levels = [True] * NUM_LEVELS
        self.locked_levels[0] = False
        self.total_reward = 0.0
        self.level = 0
        self.is_new_episode = False
        self.unlock_levels()

    # -- per-level bookkeeping ---------------------------------------------
    def start_episode(self):
        s = self.scores[self.level]
        if len(s) == 0:
            self.scores[self.level] = [0] * self.min_tries_for_avg
        else:
            s.insert(0, 0)
            self.scores[self.level] = s[: self.min_tries_for_avg]
        self.is_new_episode = True

    def standard_reward(self, episode_reward: float) -> float:
        lo = float(DOOM_SETTINGS[self.level][MIN_SCORE])
        tgt = float(DOOM_SETTINGS[self.level][TARGET_SCORE])
        hi = lo + (tgt - lo) / 0.99
        r = round(1000 * (episode_reward - lo) / (hi - lo), 4)
        return max(0.0, min(1000.0, r))

    def averages(self) -> List[float]:
        out = [0.0] * NUM_LEVELS
        for i in range(NUM_LEVELS):
            if self.scores[i]:
                n = min(len(self.scores[i]), self.average_over)
                out[i] = round(sum(self.scores[i][:n]) / n, 4)
        return out

    def get_total_reward(self) -> float:
        total = 0.0
        passed = 0
        for i in range(NUM_LEVELS):
            if self.scores[i]:
                n = min(len(self.scores[i]), self.average_over)
                avg = sum(self.scores[i][:n]) / n
                if avg >= 990:
                    passed += 1
                total += avg
        if passed == NUM_LEVELS:
            total += NUM_LEVELS * 50
        return round(total, 4)

    def unlock_levels(self):
        avg = self.averages()
        for i in range(NUM_LEVELS - 2, -1, -1):
            if self.locked_levels[i + 1] and avg[i] >= self.passing_grade:
                self.locked_levels[i + 1] = False

    def next_level(self) -> int:
        avg = self.averages()
        best, best_score = 0, 1001
        for i in range(NUM_LEVELS):
            if not self.locked_levels[i] and avg[i] < best_score:
                best, best_score = i, avg[i]
        return best

    def change_level(self, new_level=None):
        if new_level is not None and not self.locked_levels[new_level]:
            self.level = new_level
        else:
            self.level = self.next_level()
        return self.level

    def on_step(self, episode_total_reward: float, finished: bool) -> float:
        """Update with the engine's running episode reward; returns the step reward."""
        self.scores[self.level][0] = self.standard_reward(episode_total_reward)
        total = self.get_total_reward()
        reward = total - self.total_reward
        self.total_reward = total
        if self.is_new_episode:
            reward = self.total_reward
        self.is_new_episode = False
        if finished:
            self.unlock_levels()
        return reward
