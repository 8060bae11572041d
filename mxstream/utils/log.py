"""Logging: the reference only has slf4j-log4j12 on the runtime classpath
(pom.xml:56-69, no configuration). mxstream logs through Python ``logging`` with a log4j-like
line layout; the level comes from ``MXS_LOG_LEVEL`` (DEBUG/INFO/WARN/ERROR, default WARN) and the
C++ runtime reads the same variable (csrc/runtime.cpp ``mxs_log``)."""
from __future__ import annotations

import logging
import os
import sys

_FMT = "%(asctime)s %(levelname)-5s %(name)-32s - %(message)s"
_configured = False


def _level() -> int:
    name = os.environ.get("MXS_LOG_LEVEL", "WARN").upper()
    return {"WARN": logging.WARNING, "TRACE": logging.DEBUG}.get(name, getattr(logging, name,
                                                                             logging.WARNING))


class _StderrHandler(logging.StreamHandler):
    """Writes to the *current* sys.stderr (redirections after import are honoured)."""

    def emit(self, record):
        self.stream = sys.stderr
        super().emit(record)


def get_logger(name: str) -> logging.Logger:
    global _configured
    root = logging.getLogger("mxstream")
    if not _configured:
        h = _StderrHandler(sys.stderr)
        h.setFormatter(logging.Formatter(_FMT))
        root.addHandler(h)
        root.setLevel(_level())
        root.propagate = False
        _configured = True
    return root.getChild(name) if not name.startswith("mxstream") else logging.getLogger(name)


def set_level(level: str) -> None:
    os.environ["MXS_LOG_LEVEL"] = level
    get_logger("mxstream").setLevel(_level())
    logging.getLogger("mxstream").setLevel(_level())
