"""CPU lint of the Python package: every name a function loads is bound
somewhere (module scope, an enclosing function, its own scope, an import,
or builtins) -- catches a missing import before a GPU run does."""

import ast
import builtins
import glob
import os

import pytest

from conftest import ROOT

FILES = sorted(glob.glob(os.path.join(ROOT, "gsplat-triton_amd", "gsplat_hip", "*.py"))) + \
    [os.path.join(ROOT, "bench.py"), os.path.join(ROOT, "__graft_entry__.py")]


def _bound(node):
    """Names bound anywhere inside `node` (assignments, defs, imports, args,
    comprehension targets, except-as, with-as, global/nonlocal)."""
    out = set()
    for n in ast.walk(node):
        if isinstance(n, ast.Name) and isinstance(n.ctx, (ast.Store, ast.Del)):
            out.add(n.id)
        elif isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            out.add(n.name)
        elif isinstance(n, (ast.Import, ast.ImportFrom)):
            for a in n.names:
                out.add((a.asname or a.name).split(".")[0])
        elif isinstance(n, ast.arg):
            out.add(n.arg)
        elif isinstance(n, ast.ExceptHandler) and n.name:
            out.add(n.name)
        elif isinstance(n, (ast.Global, ast.Nonlocal)):
            out.update(n.names)
    return out


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f) for f in FILES])
def test_no_undefined_names(path):
    tree = ast.parse(open(path).read(), path)
    known = _bound(tree) | set(dir(builtins)) | {"__file__", "__name__", "__doc__"}
    missing = sorted({n.id for n in ast.walk(tree)
                      if isinstance(n, ast.Name) and isinstance(n.ctx, ast.Load)
                      and n.id not in known})
    assert not missing, f"{os.path.basename(path)}: undefined names {missing}"
