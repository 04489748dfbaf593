"""Reference-API compatibility surface.

A user of ``jan-hofmeier/pathnet-gym`` imports flat modules (``pathnet``,
``game_ac_network``, ``a3c_training_thread``, ``rmsprop_applier``,
``input_data``, ``constants``, ``game_state``).  This package exposes the same
names with the same call shapes, implemented on this framework's pieces
(flat parameter store, TF-semantics RMSProp, replicated GA).  It is the
migration path, not the fast path: the population-parallel HIP engine
(``algo/trainer.py`` + ``runtime/engine.py``) is what the benchmarks run.

TF-session plumbing (``sess``, placeholders, summary ops) has no meaning
without TensorFlow; those positional arguments are accepted and ignored so
that reference call sites keep working unchanged.
"""
from . import constants, pathnet  # noqa: F401
