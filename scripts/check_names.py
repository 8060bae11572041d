"""Lint for Python modules (no linter in this image):

* undefined globals: names a function reads that are bound neither in the function (any scope
  inside it), nor at module level, nor as builtins -- the NameErrors a module split would leave
  for a code path no test reaches;
* blank-line debris: runs of three or more blank lines (what a mechanical split leaves behind).

    python scripts/check_names.py mxstream/runtime/window_operator.py [...]
"""
import ast
import builtins
import sys


def bound_in(node) -> set:
    out = set()
    for n in ast.walk(node):
        if isinstance(n, ast.Name) and isinstance(n.ctx, (ast.Store, ast.Del)):
            out.add(n.id)
        elif isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            out.add(n.name)
            if not isinstance(n, ast.ClassDef):
                a = n.args
                for arg in a.posonlyargs + a.args + a.kwonlyargs:
                    out.add(arg.arg)
                if a.vararg:
                    out.add(a.vararg.arg)
                if a.kwarg:
                    out.add(a.kwarg.arg)
        elif isinstance(n, ast.Lambda):
            a = n.args
            for arg in a.posonlyargs + a.args + a.kwonlyargs:
                out.add(arg.arg)
            if a.vararg:
                out.add(a.vararg.arg)
            if a.kwarg:
                out.add(a.kwarg.arg)
        elif isinstance(n, (ast.Import, ast.ImportFrom)):
            for al in n.names:
                out.add((al.asname or al.name).split(".")[0])
        elif isinstance(n, ast.ExceptHandler) and n.name:
            out.add(n.name)
        elif isinstance(n, (ast.Global, ast.Nonlocal)):
            out.update(n.names)
    return out


def check(path: str) -> list[str]:
    tree = ast.parse(open(path).read(), path)
    module = set(dir(builtins)) | {"__file__", "__name__", "__doc__"}
    for n in tree.body:
        module |= bound_in(n) if not isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef,
                                                    ast.ClassDef)) else {n.name}
    bad = []

    def visit_fn(fn, outer: set):
        local = outer | bound_in(fn)
        for n in ast.walk(fn):
            if isinstance(n, ast.Name) and isinstance(n.ctx, ast.Load) and n.id not in local \
                    and n.id not in module:
                bad.append(f"{path}:{n.lineno}: undefined name {n.id!r} in {fn.name}")

    def visit_body(body):  # top-level functions and methods (closures: their outer scope)
        for n in body:
            if isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef)):
                visit_fn(n, set())
            elif isinstance(n, ast.ClassDef):
                visit_body(n.body)

    visit_body(tree.body)
    return sorted(set(bad))


def blank_runs(path: str, limit: int = 3) -> list[str]:
    """Runs of `limit` or more consecutive blank lines."""
    bad, run = [], 0
    lines = open(path).read().split("\n")
    for i, line in enumerate(lines + ["x"], 1):
        if line.strip() == "" and i <= len(lines):
            run += 1
            continue
        if run >= limit and i <= len(lines):
            bad.append(f"{path}:{i - run}: {run} blank lines in a row")
        run = 0
    return bad


if __name__ == "__main__":
    problems = [p for f in sys.argv[1:] for p in check(f) + blank_runs(f)]
    print("\n".join(problems) if problems else "ok")
    sys.exit(1 if problems else 0)
