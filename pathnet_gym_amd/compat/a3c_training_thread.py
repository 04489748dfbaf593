"""``A3CTrainingThread``: one reference-style actor-learner (``a3c_training_thread.py:26-245``).

Drop-in for the reference worker loop: ``set_training_stage`` builds the
``GameState`` (seed 113*task_index, ROMZ[stage], no_op_max=ACTION_SIZEZ[stage],
:75-81), ``process()`` runs up to LOCAL_T_MAX steps with host categorical
sampling, n-step returns with reward clip [-1,1] (:155-180), computes the
loss gradient with autograd and applies only the variables whose
``get_vars_idx()`` is 1 (frozen modules excluded, :190-216), prints the
"### Performance" line every PERFORMANCE_LOG_INTERVAL local steps on worker 0
(:236-241) and returns the number of local steps taken.

The episode score that the reference writes into PS variables
(``score_ops`` / ``score_set_ops``, :145-146) is delivered by calling
``score_set_ops(score)`` / ``score_ops(score)`` if they are callables, or by
storing into ``score_set_ops[task_index]`` if it is an indexable array.
Everything TF-specific (``sess``, summary writer/op, placeholders) is ignored.

This is the one-agent, host-driven API kept for migration; the batched
on-device population engine is ``algo/trainer.py``.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from ..config import ACTION_SIZEZ, ENTROPY_BETA, GAMMA, LOCAL_T_MAX, PERFORMANCE_LOG_INTERVAL, ROMZ
from ..envs.game_state import GameState
from .game_ac_network import GameACPathNetLSTMNetwork, GameACPathNetNetwork

LOG_INTERVAL = 100


def _deliver(sink, task_index, value):
    if sink is None:
        return
    if callable(sink):
        sink(value)
    else:
        try:
            sink[task_index] = value
        except (TypeError, IndexError, KeyError):
            pass


class A3CTrainingThread:
    def __init__(self, thread_index, global_network, training_stage, initial_learning_rate, learning_rate_input,
                 grad_applier, max_global_time_step, device="cpu", FLAGS="", task_index="", use_lstm=None,
                 romz=None, game_device="cpu"):
        print("Initializing worker #{}".format(task_index))
        self.training_stage = training_stage
        self.thread_index = thread_index
        self.task_index = task_index if task_index != "" else 0
        self.learning_rate_input = learning_rate_input
        self.max_global_time_step = max_global_time_step
        self.romz = list(romz or ROMZ)
        self.game_device = game_device
        if use_lstm is None:
            use_lstm = bool(getattr(FLAGS, "use_lstm", False)) if FLAGS not in (None, "") else \
                isinstance(global_network, GameACPathNetLSTMNetwork)
        self.use_lstm = use_lstm
        cls = GameACPathNetLSTMNetwork if use_lstm else GameACPathNetNetwork
        store = global_network.store if global_network is not None else None
        self.local_network = cls(training_stage, thread_index, device, FLAGS, store=store)
        self.local_network.prepare_loss(ENTROPY_BETA)
        self.grad_applier = grad_applier
        self.local_t = 0
        self.initial_learning_rate = initial_learning_rate
        self.episode_reward = 0
        self.prev_local_t = 0
        self.start_time = time.time()
        self.game_state = None
        self.rng = np.random

    def set_training_stage(self, training_stage):
        self.training_stage = training_stage
        self.local_network.set_training_stage(training_stage)
        print("Setting training task to:  " + self.romz[training_stage] + ", with action size: "
              + str(ACTION_SIZEZ[training_stage]))
        if self.game_state is not None:
            self.game_state.close_env()
        self.game_state = GameState(113 * int(self.task_index), self.romz[training_stage], display=False,
                                    no_op_max=ACTION_SIZEZ[training_stage], task_index=self.task_index,
                                    device=self.game_device)

    def _anneal_learning_rate(self, global_time_step):
        lr = self.initial_learning_rate * (self.max_global_time_step - global_time_step) / self.max_global_time_step
        return max(lr, 0.0)

    def choose_action(self, pi_values):
        p = np.asarray(pi_values, np.float64)
        return int(self.rng.choice(len(p), p=p / p.sum()))

    def set_start_time(self, start_time):
        self.start_time = start_time

    def process(self, sess=None, global_t=0, summary_writer=None, summary_op=None, score_input=None, score_ph=None,
                score_ops=None, geopath=None, FLAGS=None, score_set_ph=None, score_set_ops=None):
        if self.game_state is None:
            self.set_training_stage(self.training_stage)
        net = self.local_network
        if geopath is not None:
            net.set_geopath(geopath)
        states, actions, rewards, values = [], [], [], []
        terminal_end = False
        start_local_t = self.local_t
        start_lstm_state = net.lstm_state_out if self.use_lstm else None
        for _ in range(LOCAL_T_MAX):
            pi_, value_ = net.run_policy_and_value(self.game_state.s_t)
            action = self.choose_action(pi_)
            states.append(self.game_state.s_t)
            actions.append(action)
            values.append(value_)
            self.game_state.process(action)
            reward, terminal = self.game_state.reward, self.game_state.terminal
            self.episode_reward += reward
            rewards.append(float(np.clip(reward, -1, 1)))
            self.local_t += 1
            self.game_state.update()
            if terminal:
                terminal_end = True
                _deliver(score_ops, self.task_index, self.episode_reward)
                _deliver(score_set_ops, self.task_index, self.episode_reward)
                self.episode_reward = 0
                self.game_state.reset()
                if self.use_lstm:
                    net.reset_state()
                break
        R = 0.0 if terminal_end else net.run_value(self.game_state.s_t)
        A = max(ACTION_SIZEZ)
        batch_a = np.zeros((len(actions), A), np.float32)
        batch_td = np.zeros(len(actions), np.float32)
        batch_R = np.zeros(len(actions), np.float32)
        for i in reversed(range(len(actions))):
            R = rewards[i] + GAMMA * R
            batch_td[i] = R - values[i]
            batch_a[i, actions[i]] = 1.0
            batch_R[i] = R
        lr = self._anneal_learning_rate(global_t)
        flat = net.store.flat
        flat.grad = None
        loss = net.loss(np.stack(states), batch_a, batch_td, batch_R, start_lstm_state)
        loss.backward()
        grads = net.grads_for(flat.grad, full=True)
        vars_all = net.all_vars()
        idx = net.get_vars_idx()
        sel_v = [v for v, k in zip(vars_all, idx) if k == 1]
        sel_g = [g for g, k in zip(grads, idx) if k == 1]
        self.grad_applier.apply_gradients(sel_v, sel_g, learning_rate=lr)
        flat.grad = None
        if int(self.task_index or 0) == 0 and self.local_t - self.prev_local_t >= PERFORMANCE_LOG_INTERVAL:
            self.prev_local_t += PERFORMANCE_LOG_INTERVAL
            elapsed = time.time() - self.start_time
            sps = global_t / max(elapsed, 1e-9)
            print("### Performance : {} STEPS in {:.0f} sec. {:.0f} STEPS/sec. {:.2f}M STEPS/hour".format(
                global_t, elapsed, sps, sps * 3600 / 1000000.))
        return self.local_t - start_local_t
