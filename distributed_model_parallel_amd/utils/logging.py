"""Metrics logging.

The reference appends one text line per epoch to ``./log/512.txt`` /
``./log/data_para_512.txt`` (``model_parallel.py:119-125``,
``data_parallel.py:166-171``) without creating ``./log`` first (defect 7)
and only from rank 0.  :class:`MetricsLogger` writes the same human-readable
line (same keys) AND a structured JSONL record per rank, creating
directories as needed; images/sec, step time and comm/compute breakdowns go
in the JSON record.
"""
from __future__ import annotations

import json
import os
import sys
import time
from typing import Any, Dict, Optional


def reference_line(epoch: int, rec: Dict[str, Any]) -> str:
    """``step:E  loss_train:..  acc1_train:..  loss_val:..  acc1_val:..[  time_per_batch:..
    time_load_perbatch:..]`` exactly in the reference's key order."""
    parts = [f"step:{epoch}"]
    for k in ("loss_train", "acc1_train", "loss_val", "acc1_val", "time_per_batch",
              "time_load_perbatch"):
        if k in rec and rec[k] is not None:
            parts.append(f"{k}:{rec[k]}")
    return "  ".join(parts)


class MetricsLogger:
    def __init__(self, log_dir: str = "./log", name: str = "train", rank: int = 0,
                 text_file: Optional[str] = None, echo: bool = True):
        self.rank = rank
        self.echo = echo and rank == 0
        os.makedirs(log_dir, exist_ok=True)
        self.jsonl_path = os.path.join(log_dir, f"{name}.rank{rank}.jsonl")
        self.text_path = os.path.join(log_dir, text_file) if (text_file and rank == 0) else None
        self.t0 = time.time()

    def log(self, epoch: int, **rec: Any) -> None:
        rec = {k: (float(v) if hasattr(v, "item") else v) for k, v in rec.items()}
        full = {"epoch": epoch, "rank": self.rank, "wall_s": round(time.time() - self.t0, 3), **rec}
        with open(self.jsonl_path, "a") as f:
            f.write(json.dumps(full) + "\n")
        if self.text_path:
            with open(self.text_path, "a") as f:
                f.write("\n" + reference_line(epoch, rec))
        if self.echo:
            print(reference_line(epoch, rec), file=sys.stdout, flush=True)

    def event(self, name: str, **rec: Any) -> None:
        with open(self.jsonl_path, "a") as f:
            f.write(json.dumps({"event": name, "rank": self.rank,
                                "wall_s": round(time.time() - self.t0, 3), **rec}) + "\n")
