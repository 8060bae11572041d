"""Source hygiene of the package (scripts/check_names.py): no undefined globals a refactor left
behind, and no runs of three or more blank lines."""
import importlib.util
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _lint():
    spec = importlib.util.spec_from_file_location("check_names", ROOT / "scripts" / "check_names.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_package_has_no_undefined_names_or_blank_runs():
    lint = _lint()
    files = sorted(str(p) for p in (ROOT / "mxstream").rglob("*.py"))
    files += [str(ROOT / "bench.py"), str(ROOT / "__graft_entry__.py")]
    problems = [p for f in files for p in lint.check(f) + lint.blank_runs(f)]
    assert not problems, "\n".join(problems)
