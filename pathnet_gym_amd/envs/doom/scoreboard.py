"""Scoreboard metadata for the Doom ids (reference ``gym_doom/__init__.py:95-387``, old gym.scoreboard API).

The reference registers one group ("doom") and one task entry per id with a
summary and a longer description for the (long gone) OpenAI Gym scoreboard.
Here the same add_group / add_task calls fill a plain registry that tools
(CLI ``info``, docs) can read; the summaries are short paraphrases.
"""
from __future__ import annotations

from typing import Dict

GROUPS: Dict[str, dict] = {}
TASKS: Dict[str, dict] = {}


def add_group(id: str, name: str, description: str = "") -> None:   # noqa: A002  (gym signature)
    GROUPS[id] = {"name": name, "description": description}


def add_task(id: str, group: str, summary: str = "", description: str = "", contributor: str = "",
             **extra) -> None:   # noqa: A002
    if group not in GROUPS:
        raise KeyError(f"unknown scoreboard group {group!r}")
    TASKS[id] = {"group": group, "summary": summary, "description": description, "contributor": contributor, **extra}


add_group("doom", "Doom", "First-person 3D navigation and combat scenarios driven through the ViZDoom engine.")
_SUMMARIES = {
    "gym_doom/meta-Doom-v0": "Curriculum over the nine levels; reward = change of the standardised total score.",
    "gym_doom/DoomBasic-v0": "Shoot the single monster in a small room as quickly as possible.",
    "gym_doom/DoomCorridor-v0": "Run down a corridor past shooting monsters to reach the vest.",
    "gym_doom/DoomDefendCenter-v0": "Stand in the centre and kill approaching monsters with limited ammo.",
    "gym_doom/DoomDefendLine-v0": "Hold a line against monsters attacking from the far side of the room.",
    "gym_doom/DoomHealthGathering-v0": "Survive on an acid floor by picking up medkits.",
    "gym_doom/DoomMyWayHome-v0": "Find the vest somewhere in a maze of rooms.",
    "gym_doom/DoomPredictPosition-v0": "Hit a moving monster with a slow rocket by leading the shot.",
    "gym_doom/DoomTakeCover-v0": "Dodge fireballs from monsters you cannot attack.",
    "gym_doom/DoomDeathmatch-v0": "Kill as many monsters as possible in a large arena with weapons and items.",
}
for _id, _s in _SUMMARIES.items():
    add_task(_id, "doom", summary=_s)
