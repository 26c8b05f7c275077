"""Shared CLI plumbing: Go-flag-compatible argument parsing and output helpers.

REF binaries use Go's ``flag`` package, which accepts ``-flag``, ``--flag``, ``-flag=v``
and ``--flag=v`` and ``--version``/``version`` as the sole argument
(e.g. REF cmd/agent/main.go:329-332). ``GoFlags`` mirrors that surface on argparse.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
from typing import IO, Any, Callable, List, Optional, Sequence, Tuple

from .. import __version__


def is_version_request(argv: Sequence[str]) -> bool:
    return len(argv) == 1 and argv[0] in ("--version", "version", "-version")


class GoFlags(argparse.ArgumentParser):
    """argparse with Go flag spelling: every ``--name`` is also accepted as ``-name``."""

    def __init__(self, prog: str, description: str = ""):
        super().__init__(prog=prog, description=description, allow_abbrev=False)

    def flag(self, name: str, default: Any = None, help: str = "", type: Optional[Callable] = None,
             choices: Optional[Sequence[Any]] = None, dest: Optional[str] = None) -> None:
        kw = {"default": default, "help": help, "dest": dest or name.replace("-", "_")}
        if isinstance(default, bool) and type is None:
            kw["type"] = parse_bool
            kw["nargs"] = "?"
            kw["const"] = True
        else:
            kw["type"] = type or (default.__class__ if default is not None else str)
        if choices is not None:
            kw["choices"] = choices
        self.add_argument(f"--{name}", f"-{name}", **kw)


def parse_bool(v: str) -> bool:
    s = str(v).strip().lower()
    if s in ("1", "t", "true", "yes", "y", "on"):
        return True
    if s in ("0", "f", "false", "no", "n", "off", ""):
        return False
    raise argparse.ArgumentTypeError(f"invalid boolean value {v!r}")


def split_csv(raw: str) -> List[str]:
    return [p.strip() for p in (raw or "").split(",") if p.strip()]


def ensure_parent(path: str) -> None:
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)


def open_output(path: str) -> Tuple[IO[str], Callable[[], None]]:
    """'-' = stdout (REF openOutput, cmd/attributor/main.go:227-241)."""
    if path == "-":
        return sys.stdout, lambda: sys.stdout.flush()
    ensure_parent(path)
    fh = open(path, "w", encoding="utf-8")
    return fh, fh.close


def write_json(path: str, payload: Any) -> None:
    ensure_parent(path)
    with open(path, "w", encoding="utf-8") as fh:
        json.dump(payload, fh, indent=2)


def jsonl_line(obj: Any) -> str:
    d = obj.to_dict() if hasattr(obj, "to_dict") else obj
    return json.dumps(d, separators=(",", ":")) + "\n"


def eprint(*a) -> None:
    print(*a, file=sys.stderr, flush=True)


def print_version() -> int:
    print(__version__)
    return 0


def project_root() -> str:
    """Repository root (the directory holding config/ and docs/) -- REF projectRoot."""
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(os.path.dirname(here))
    return root
