"""Logging set-up with the reference's environment contract (bmi/logger.py).

Environment variables honoured (logger.py:22-25): NGEN_EWTS_LOGGING,
NGEN_LOG_FILE_PATH, TOPOFLOW_GLACIER_LOGLEVEL, TOPOFLOW_GLACIER_LOGFILEPATH.
The reference's extra level names SEVERE and FATAL are registered.  When a log
file cannot be opened, output goes to stdout, as the reference ends up doing.
"""

from __future__ import annotations

import logging
import os
import sys

__all__ = ["logger", "configure_logging"]

MODULE_NAME = "Topoflow-Glacier"
logger = logging.getLogger(MODULE_NAME)

SEVERE = logging.ERROR + 1
FATAL = logging.CRITICAL
logging.addLevelName(SEVERE, "SEVERE")
logging.addLevelName(FATAL, "FATAL")

_configured = False


def configure_logging() -> logging.Logger:
    """Idempotent: many model instances may share a process (ngen)."""
    global _configured
    if _configured:
        return logger
    level_name = os.environ.get("TOPOFLOW_GLACIER_LOGLEVEL", "INFO").upper()
    level = logging.getLevelName(level_name)
    if not isinstance(level, int):
        level = logging.INFO
    path = None
    if os.environ.get("NGEN_EWTS_LOGGING", "").upper() == "ENABLED":
        path = os.environ.get("NGEN_LOG_FILE_PATH")
    path = path or os.environ.get("TOPOFLOW_GLACIER_LOGFILEPATH")
    handler: logging.Handler
    try:
        if path:
            os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
            handler = logging.FileHandler(path)
        else:
            raise OSError
    except OSError:
        handler = logging.StreamHandler(sys.stdout)
    handler.setFormatter(logging.Formatter(f"%(asctime)s {MODULE_NAME} %(levelname)s: %(message)s"))
    logger.handlers[:] = [handler]
    logger.setLevel(level)
    logger.propagate = False
    _configured = True
    return logger
