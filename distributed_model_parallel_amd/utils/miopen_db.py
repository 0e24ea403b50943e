"""Committed MIOpen find / perf databases for the convolutions left on MIOpen.

ResNet-50 keeps its 7x7 stem and the 3x3 data / weight gradients on MIOpen
(ops/conv_igemm.py), and the bench runs MIOpen in find mode
(``cudnn.benchmark``).  On a fresh MI355X box the first training step then
spends ~50 s timing every solver for each problem (measured: warm-up step 0
104.6 s with an empty user database vs 54.4 s with the database below; the
kernel binary cache made no difference, ``profiles/README.md`` finding 9).

Measured further (``tools/first_step.py`` with ``MIOPEN_LOG_LEVEL=5``): with
the find db seeded, MIOpen's find still *times* every applicable solver, and
~54 s of the remaining first step is the reference "naive" direct solvers
(``ConvDirectNaive{Fwd,Bwd,Wrw}``: e.g. 2.37 s per timing run of the stem's
weight gradient, 30-1000x slower than the implicit-GEMM solvers that always
win).  :func:`seed` therefore also takes them out of find's candidate list
(``MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_*=0``, unless the user set them): every
conv of the bench models has two implicit-GEMM solvers applicable (checked
against the db: ``tests/test_aux.py``).

The databases are MIOpen's own text formats (``*.ufdb.txt``: find results,
``*.udb.txt``: tuned solver parameters), produced by a bench run on MI355X and
kept under ``profiles/miopen/``.  :func:`seed` copies them into a per-rank
writable directory and points ``MIOPEN_USER_DB_PATH`` at it -- MIOpen reads the
variable when its first handle is created, so call this before the first conv.
A user-set ``MIOPEN_USER_DB_PATH`` is left alone.  Entries are keyed by the
full problem (batch, shape, layout, dtype) and MIOpen version: shapes that are
not in the file are searched as usual and nothing else changes.

  python bench.py --miopen-db refresh   # search, then write the found entries back
  DMP_MIOPEN_DB_OUT=gpurun_out/miopen python bench.py --miopen-db refresh   # ... elsewhere
"""
from __future__ import annotations

import atexit
import os
import shutil
from pathlib import Path
from typing import Optional

ROOT = Path(__file__).resolve().parents[2]
DB_DIR = ROOT / "profiles" / "miopen"
_ENV = "MIOPEN_USER_DB_PATH"
NAIVE_SOLVER_ENVS = tuple(f"MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_{d}" for d in ("FWD", "BWD", "WRW"))


def _rank_dir() -> Path:
    base = Path(os.environ.get("TMPDIR", "/tmp"))
    tag = f"{os.getuid() if hasattr(os, 'getuid') else 0}_{os.getpid()}"
    return base / f"dmp_miopen_db_{tag}"


def seed(mode: str = "use", skip_naive: bool = True) -> Optional[str]:
    """mode "use": seed from the committed db; "refresh": seed, then copy the
    (possibly grown) db back at exit; "off": MIOpen defaults.  Returns the
    directory MIOpen will use, or None when untouched.  skip_naive: drop the
    naive reference solvers from find (module docstring)."""
    if mode == "off":
        return None
    if skip_naive:
        for k in NAIVE_SOLVER_ENVS:
            os.environ.setdefault(k, "0")
    if os.environ.get(_ENV):
        return None
    if mode not in ("use", "refresh"):
        raise ValueError(f"unknown miopen db mode {mode!r}")
    d = _rank_dir()
    d.mkdir(parents=True, exist_ok=True)
    if DB_DIR.is_dir():
        for f in DB_DIR.glob("*.txt"):
            shutil.copy2(f, d / f.name)
    os.environ[_ENV] = str(d)
    if mode == "refresh":
        atexit.register(_write_back, d)
    else:
        atexit.register(shutil.rmtree, d, True)
    return str(d)


def _write_back(d: Path) -> None:
    # DMP_MIOPEN_DB_OUT: write somewhere else (e.g. gpurun_out/ on a remote box,
    # to be copied into profiles/miopen/ afterwards)
    out = Path(os.environ.get("DMP_MIOPEN_DB_OUT", str(DB_DIR)))
    out.mkdir(parents=True, exist_ok=True)
    for f in d.glob("*.txt"):
        shutil.copy2(f, out / f.name)
    shutil.rmtree(d, ignore_errors=True)
