"""Doom adapters and MetaDoom scoring (pure logic of gym_doom/, engine not required)."""
import pytest

from pathnet_gym_amd.envs import doom
from pathnet_gym_amd.envs.doom import (BoxToMultiDiscrete, DiscreteToMultiDiscrete, MetaDoomScorer, MultiDiscrete,
                                       ToBox, ToDiscrete)
from pathnet_gym_amd.envs.doom.constants import BUTTON_RANGES
from pathnet_gym_amd.envs.doom.spaces import SpaceError


def test_tables():
    assert len(doom.BUTTONS) == 43 and doom.BUTTONS[13] == "MOVE_FORWARD"
    assert len(doom.DOOM_SETTINGS) == 9 and doom.DOOM_SETTINGS[0][doom.ACTIONS] == [0, 10, 11]
    assert 33 not in doom.DOOM_SETTINGS[8][doom.ACTIONS]
    assert len(doom.GAME_VARIABLES) == 22 and len(doom.RESOLUTIONS) == 36
    assert doom.DOOM_REGISTRY["gym_doom/DoomBasic-v0"] == (0, 10000, 10.0)


def test_discrete_adapter_configs():
    md = MultiDiscrete([[0, 4], [0, 1], [0, 1]])
    d1 = DiscreteToMultiDiscrete(md)
    assert d1.n == 4 and d1(0) == [0, 0, 0] and d1(1) == [4, 0, 0] and d1(3) == [0, 0, 1]
    d2 = DiscreteToMultiDiscrete(md, [0, 2])
    assert d2.n == 3 and d2(2) == [0, 0, 1]
    d3 = DiscreteToMultiDiscrete(md, {0: [0, 0, 0], 1: [2, 1, 0]})
    assert d3.n == 2 and d3(1) == [2, 1, 0]
    with pytest.raises(SpaceError):
        DiscreteToMultiDiscrete(md, {1: [0, 0, 0]})
    with pytest.raises(SpaceError):
        DiscreteToMultiDiscrete(md, {0: [9, 0, 0]})


def test_box_adapter():
    md = MultiDiscrete([[0, 4], [0, 1], [0, 1]])
    b = BoxToMultiDiscrete(md, [2, 0])
    assert list(b.low) == [0, 0] and list(b.high) == [1, 4]
    assert b([0.7412057, 3.0174142]) == [3, 0, 1]


class FakeDoom:
    def __init__(self, level=0):
        self.level = level
        self.action_space = MultiDiscrete(BUTTON_RANGES)
        self.sent = None

    @property
    def unwrapped(self):
        return self

    def step(self, a):
        self.sent = a
        return None, 0.0, False, {}


def test_to_discrete_wrapper_configs():
    env = ToDiscrete("minimal")(FakeDoom(0))
    assert env.action_space.n == 4
    env.step(2)
    assert env.unwrapped.sent[10] == 1 and sum(env.unwrapped.sent) == 1
    assert ToDiscrete("constant-7")(FakeDoom(3)).action_space.n == 8
    assert ToDiscrete("constant-17")(FakeDoom(3)).action_space.n == 18
    assert ToDiscrete("full")(FakeDoom(3)).action_space.n == 44
    with pytest.raises(SpaceError):
        ToDiscrete("bogus")(FakeDoom(0))
    box = ToBox("minimal")(FakeDoom(7))
    box.step([0.9, 0.2])
    assert box.unwrapped.sent[10] == 1 and box.unwrapped.sent[11] == 0


def test_meta_doom_scoring():
    s = MetaDoomScorer(average_over=3, passing_grade=600, min_tries_for_avg=3)
    assert s.locked_levels == [False] + [True] * 8
    # basic: min -485, target 10 -> max = -485 + 495/0.99 = 15; 10 -> 990
    assert s.standard_reward(10) == 990.0 and s.standard_reward(-1000) == 0.0 and s.standard_reward(100) == 1000.0
    s.start_episode()
    assert s.scores[0] == [0, 0, 0]
    r = s.on_step(10.0, finished=True)        # first step of an episode returns the total
    assert r == s.total_reward == round(990 / 3, 4)
    for _ in range(2):
        s.start_episode()
        s.on_step(10.0, finished=True)
    assert s.averages()[0] == 990.0
    assert s.locked_levels[1] is False                        # unlocked at >= passing grade
    assert s.next_level() == 1                                # lowest unlocked average
    s.level = 1
    s.start_episode()
    s.on_step(-120, finished=False)
    assert s.scores[1][0] == 0.0


def test_engine_gating():
    with pytest.raises(doom.DependencyNotInstalled):
        doom.make_doom("gym_doom/DoomBasic-v0")


def test_scoreboard_metadata_covers_every_id():
    from pathnet_gym_amd.envs.doom import DOOM_REGISTRY, scoreboard
    assert set(scoreboard.TASKS) == set(DOOM_REGISTRY)
    assert all(t["group"] == "doom" and t["summary"] for t in scoreboard.TASKS.values())


def test_generated_scenario_configs_match_reference_settings(tmp_path):
    """The nine scenario .cfg files (gym_doom/assets/*.cfg) generated from one table."""
    from pathnet_gym_amd.envs.doom import scenarios as sc
    from pathnet_gym_amd.envs.doom.constants import ALLOWED_ACTIONS, BUTTONS, DOOM_SETTINGS
    d = sc.write_assets(str(tmp_path))
    for li, row in enumerate(DOOM_SETTINGS):
        cfg = sc.parse_cfg(open(f"{d}/{row[0]}").read())
        assert cfg["screen_format"] == "BGR24" and cfg["sound_enabled"] == "false"
        assert len(cfg["available_game_variables"]) == 22
        # the level's allowed buttons (doom_env.py:33-44) are exactly the config's buttons
        names = [BUTTONS[i].replace("ALT_ATTACK", "ALTATTACK") for i in ALLOWED_ACTIONS[li]]
        assert sorted(cfg["available_buttons"]) == sorted(names), row[0]
    basic = sc.parse_cfg(sc.render_cfg("basic.cfg"))
    assert basic["living_reward"] == "-10" and basic["episode_start_time"] == "14" and basic["episode_timeout"] == "350"
    assert basic["available_buttons"] == ["ATTACK", "MOVE_RIGHT", "MOVE_LEFT"]
    assert sc.parse_cfg(sc.render_cfg("deathmatch.cfg"))["episode_timeout"] == "6300"
    assert sc.parse_cfg(sc.render_cfg("health_gathering.cfg"))["death_penalty"] == "100"
