"""Load numba 0.54 (conda python3.9) against numpy 1.26 — oracle/fixture generation only.

Recipe from SURVEY.md Appendix A: stub numba.np.ufunc._internal (C extension ABI-broken against
numpy 1.26), spoof numpy's version during import, alias np.MachAr.  Run scripts with
    NUMBA_CACHE_DIR=/tmp/numba_cache /opt/conda/bin/python3.9 -W ignore <script>
"""
import sys
import types

import numpy as np

_real = np.__version__
np.__version__ = "1.20.3"
_m = types.ModuleType("numba.np.ufunc._internal")


class _DUFunc(object):
    def __init__(self, *a, **k):
        pass


def _fromfunc(*a, **k):
    raise NotImplementedError


_m._DUFunc = _DUFunc
_m.PyUFunc_None = -1
_m.PyUFunc_Zero = 0
_m.PyUFunc_One = 1
_m.PyUFunc_ReorderableNone = -2
_m.fromfunc = _fromfunc
sys.modules["numba.np.ufunc._internal"] = _m
try:
    from numpy.core._machar import MachAr as _MA
except Exception:  # pragma: no cover
    class _MA(object):
        pass
np.MachAr = _MA
import numba  # noqa: E402,F401

np.__version__ = _real


def load_reference(path="/root/reference/Anis_TTF_rays.py", pad_rows=256):
    """Exec the reference with the 'padded' stage-1 arrays and cache=False."""
    import ast

    class Pad(ast.NodeTransformer):
        def visit_Assign(self, node):
            self.generic_visit(node)
            t = node.targets[0]
            if isinstance(t, ast.Name) and t.id in ("ttn1", "nsts1") and isinstance(node.value, (ast.Call, ast.UnaryOp)):
                src = ast.unparse(node.value) if hasattr(ast, "unparse") else ""
                if "veln1" in src:
                    if t.id == "ttn1" and "zeros" in src:
                        e = "np.zeros((veln1.shape[0] + %d, veln1.shape[1]))[:veln1.shape[0]]" % pad_rows
                    elif t.id == "nsts1" and "ones_like" in src:
                        e = ("(-np.ones((veln1.shape[0] + %d, veln1.shape[1]), dtype=veln1.dtype))"
                             "[:veln1.shape[0]]" % pad_rows)
                    else:
                        return node
                    node.value = ast.copy_location(ast.parse(e, mode="eval").body, node.value)
                    PATCHED.append((t.id, node.lineno))
            return node

        def visit_Call(self, node):
            self.generic_visit(node)
            if getattr(node.func, "id", None) == "njit":
                for kw in node.keywords:
                    if kw.arg == "cache":
                        kw.value = ast.copy_location(ast.Constant(value=False), kw.value)
            return node

    PATCHED = []
    with open(path) as fh:
        tree = ast.parse(fh.read())
    tree = ast.fix_missing_locations(Pad().visit(tree))
    mod = types.ModuleType("Anis_TTF_rays_padded")
    sys.modules["Anis_TTF_rays_padded"] = mod
    exec(compile(tree, path, "exec"), mod.__dict__)
    mod.tqdm_disable = True
    mod._PATCHED = PATCHED
    return mod
