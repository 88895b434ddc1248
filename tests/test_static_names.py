"""Static check (CPU): every name a function of bench.py / the package loads is bound somewhere it
can see -- its own scope, an enclosing function, the module, or the builtins.  bench.py's GPU-only
legs never run here, so a stray name there (round 4: `build_rec` in the config-4 line) would only
surface as a NameError on the GPU box."""
import ast
import builtins
import glob
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILES = [os.path.join(ROOT, "bench.py"), os.path.join(ROOT, "__graft_entry__.py")] + sorted(
    glob.glob(os.path.join(ROOT, "kmer_hasher_amd", "*.py")))


def _bound(node) -> set:
    """Names bound directly in this scope (not inside nested functions / classes / lambdas)."""
    out = set()
    if isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef, ast.Lambda)):
        a = node.args
        for x in a.posonlyargs + a.args + a.kwonlyargs:
            out.add(x.arg)
        if a.vararg:
            out.add(a.vararg.arg)
        if a.kwarg:
            out.add(a.kwarg.arg)
    body = node.body if isinstance(node.body, list) else [node.body]
    stack = list(body)
    while stack:
        n = stack.pop()
        if isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            out.add(n.name)
            stack.extend(n.decorator_list)
            continue
        if isinstance(n, ast.Lambda):
            continue
        if isinstance(n, ast.Name) and isinstance(n.ctx, (ast.Store, ast.Del)):
            out.add(n.id)
        elif isinstance(n, (ast.Import, ast.ImportFrom)):
            for al in n.names:
                out.add((al.asname or al.name).split(".")[0])
        elif isinstance(n, (ast.Global, ast.Nonlocal)):
            out.update(n.names)
        elif isinstance(n, ast.ExceptHandler) and n.name:
            out.add(n.name)
        elif isinstance(n, ast.arg):
            out.add(n.arg)
        stack.extend(ast.iter_child_nodes(n))
    return out


def _loads(node) -> list:
    """(name, line) loaded directly in this scope, comprehension targets counted as bound."""
    out = []
    body = node.body if isinstance(node.body, list) else [node.body]
    stack = list(body)
    comp_bound = set()
    while stack:
        n = stack.pop()
        if isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef, ast.Lambda)):
            if not isinstance(n, ast.Lambda):
                stack.extend(n.decorator_list)
                if not isinstance(n, ast.ClassDef):
                    stack.extend(n.args.defaults + n.args.kw_defaults)
            continue
        if isinstance(n, ast.comprehension):
            for t in ast.walk(n.target):
                if isinstance(t, ast.Name):
                    comp_bound.add(t.id)
        if isinstance(n, ast.Name) and isinstance(n.ctx, ast.Load):
            out.append((n.id, n.lineno))
        stack.extend(x for x in ast.iter_child_nodes(n) if x is not None)
    return [(nm, ln) for nm, ln in out if nm not in comp_bound]


def _check(tree) -> list:
    bad = []
    mod = _bound(tree) | set(dir(builtins)) | {"__file__", "__name__"}

    def visit(fn, outer):
        seen = outer | _bound(fn)
        for nm, ln in _loads(fn):
            if nm not in seen:
                bad.append((nm, ln))
        for n in ast.walk(fn):
            if n is not fn and isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.Lambda)):
                # only direct children functions: deeper ones are visited from their parent
                if _parent_fn.get(id(n)) is fn:
                    visit(n, seen)

    _parent_fn = {}

    def index(node, fn):
        for c in ast.iter_child_nodes(node):
            if isinstance(c, (ast.FunctionDef, ast.AsyncFunctionDef, ast.Lambda)):
                _parent_fn[id(c)] = fn
                index(c, c)
            else:
                index(c, fn)

    index(tree, None)
    for n in ast.walk(tree):
        if isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.Lambda)) and \
                _parent_fn.get(id(n)) is None:
            visit(n, mod | _class_names(tree))
    return bad


def _class_names(tree) -> set:
    return {n.name for n in ast.walk(tree) if isinstance(n, ast.ClassDef)}


@pytest.mark.parametrize("path", FILES, ids=lambda p: os.path.relpath(p, ROOT))
def test_no_unbound_names(path):
    tree = ast.parse(open(path).read(), path)
    bad = _check(tree)
    assert not bad, f"{os.path.relpath(path, ROOT)}: names loaded but never bound: {bad}"
