"""Every ``_lib.call("name", ...)`` site passes exactly as many arguments as the ctypes table declares.

A wrong count only fails when the call runs on a GPU; this catches it on the CPU.
"""
import ast
import glob
import os

from pathnet_gym_amd.ops import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_lib_call_sites_match_ctypes_signatures():
    sigs = _lib._SIGS
    checked, bad = 0, []
    for f in glob.glob(os.path.join(ROOT, "pathnet_gym_amd", "**", "*.py"), recursive=True):
        tree = ast.parse(open(f).read())
        for n in ast.walk(tree):
            if not (isinstance(n, ast.Call) and getattr(n.func, "attr", None) == "call" and n.args
                    and isinstance(n.args[0], ast.Constant) and n.args[0].value in sigs):
                continue
            if any(isinstance(a, ast.Starred) for a in n.args):
                continue
            checked += 1
            name = n.args[0].value
            if len(n.args) - 1 != len(sigs[name]):
                bad.append((os.path.relpath(f, ROOT), n.lineno, name, len(n.args) - 1, len(sigs[name])))
    assert checked > 20
    assert not bad, bad
