import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "sisap23-laion-challenge-learned-index_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no HIP device in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


# ---------------------------------------------------------------------------
# tie-window accounting (VERDICT r2 "weak 1a"): every oracle.compare_lists call
# of every test records how many rows matched only through the tie window
# (ids differing inside a run of distances tied within `tie`); the totals per
# test are printed at the end of the run and, with LMI_TIE_REPORT=<path>,
# written as JSON
# ---------------------------------------------------------------------------
_TIES = {}
_BYMODE = {}
_CURRENT = ["<collection>"]


def _mode_key(nodeid: str, tie: float):
    """(side, arithmetic, checked against) of one compare_lists call:
    side "product" for the GPU tests, "oracle" for the CPU oracle-vs-reference
    tests; arithmetic "split" for float32 data that is not fp16-exact (the
    split mode, r5 fixtures), else "float64" (tie 1e-12) or "float32"; the
    reference's own fixtures (golden tests) or the oracle."""
    side = "product" if "test_gpu_" in nodeid else "oracle"
    split = "split" in nodeid or "golden_r5" in nodeid or "[x_" in nodeid
    arith = ("split-" if split else "") + ("float64" if tie <= 1e-12 else "float32")
    against = "reference fixtures" if ("golden" in nodeid or "reference" in nodeid) else "oracle"
    return side, arith, against


def _install_tie_accounting():
    import lmi_oracle as O
    if getattr(O.compare_lists, "_counted", False):
        return
    inner = O.compare_lists

    def compare_lists(*a, stats=None, **kw):
        st = {}
        bad = inner(*a, stats=st, **kw)
        if stats is not None:
            stats.update(st)
        acc = _TIES.setdefault(_CURRENT[0], {"calls": 0, "rows": 0, "mismatched": 0, "tie_rows": 0,
                                             "exact_tie_rows": 0, "tie": set()})
        acc["calls"] += 1
        for key in ("rows", "mismatched", "tie_rows", "exact_tie_rows"):
            acc[key] += st[key]
        acc["tie"].add(st["tie"])
        if "sharp" in _CURRENT[0]:
            return bad  # (the sharpness tests count disagreements on purpose)
        mk = _mode_key(_CURRENT[0], st["tie"])
        bm = _BYMODE.setdefault(mk, {"rows": 0, "tie_rows": 0, "exact_tie_rows": 0})
        for key in ("rows", "tie_rows", "exact_tie_rows"):
            bm[key] += st[key]
        return bad

    compare_lists._counted = True
    O.compare_lists = compare_lists


_install_tie_accounting()


def pytest_runtest_setup(item):
    _CURRENT[0] = item.nodeid


def pytest_terminal_summary(terminalreporter):
    if not _TIES:
        return
    rows = sum(v["rows"] for v in _TIES.values())
    ties = sum(v["tie_rows"] for v in _TIES.values())
    terminalreporter.write_sep("-", f"tie window: {ties} of {rows} compared rows matched only "
                                    f"through it")
    for name, v in sorted(_TIES.items()):
        if v["tie_rows"]:
            terminalreporter.write_line(f"  {name}: {v['tie_rows']}/{v['rows']} rows "
                                        f"({v['exact_tie_rows']} exact ties), tie={sorted(v['tie'])}")
    terminalreporter.write_line("  by (side, arithmetic, checked against): rows / tie-window rows "
                                "(exact ties, non-exact)")
    for mk, v in sorted(_BYMODE.items()):
        terminalreporter.write_line(f"    {' / '.join(mk)}: {v['rows']} / {v['tie_rows']} "
                                    f"({v['exact_tie_rows']}, {v['tie_rows'] - v['exact_tie_rows']})")
    path = os.environ.get("LMI_TIE_REPORT")
    if path:
        out = {k: {**v, "tie": sorted(v["tie"])} for k, v in _TIES.items()}
        out["_by_mode"] = {" / ".join(mk): v for mk, v in sorted(_BYMODE.items())}
        with open(path, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)
