"""Compiled JSON-schema validator (the draft 2020-12 subset the contracts use).

REF validates every event by re-reading and re-compiling the schema file on each call
(pkg/schema/validator.go:13-41) -- on the agent hot path that is one file read + one
schema compile per event. Here a schema is compiled ONCE into a tree of closures and
cached; validating a payload is a single walk with no allocation beyond the error list.

Supported keywords: type (single or list), enum, properties, required,
additionalProperties (bool or schema), items, minItems, minimum, maximum, minLength,
format (date-time). ``default``/``title``/``$id``/``$schema`` are annotations.
"""

from __future__ import annotations

import json
import math
import re
import threading
from typing import Any, Callable, Dict, List, Optional

from . import schemas as _schemas

Checker = Callable[[Any, str, List[str]], None]

_RFC3339 = re.compile(
    r"^\d{4}-\d{2}-\d{2}[Tt]\d{2}:\d{2}:\d{2}(\.\d+)?([Zz]|[+-]\d{2}:\d{2})$"
)


class ValidationError(ValueError):
    def __init__(self, errors: List[str]):
        super().__init__("payload failed schema validation: " + "; ".join(errors))
        self.errors = errors


def _is_type(value: Any, t: str) -> bool:
    if t == "string":
        return isinstance(value, str)
    if t == "boolean":
        return isinstance(value, bool)
    if t == "integer":
        if isinstance(value, bool):
            return False
        if isinstance(value, int):
            return True
        return isinstance(value, float) and math.isfinite(value) and value.is_integer()
    if t == "number":
        return isinstance(value, (int, float)) and not isinstance(value, bool)
    if t == "object":
        return isinstance(value, dict)
    if t == "array":
        return isinstance(value, (list, tuple))
    if t == "null":
        return value is None
    raise ValueError(f"unsupported schema type {t!r}")


def _compile(node: Dict[str, Any]) -> Checker:
    checks: List[Checker] = []

    types = node.get("type")
    if types is not None:
        tlist = [types] if isinstance(types, str) else list(types)

        def check_type(v, path, errs, tlist=tlist):
            if not any(_is_type(v, t) for t in tlist):
                errs.append(f"{path or '(root)'}: invalid type, expected {'/'.join(tlist)}")
        checks.append(check_type)

    if "enum" in node:
        allowed = list(node["enum"])

        def check_enum(v, path, errs, allowed=allowed):
            if not any(v == a and type(v) is type(a) for a in allowed):
                errs.append(f"{path or '(root)'}: must be one of {allowed}")
        checks.append(check_enum)

    if "minimum" in node or "maximum" in node:
        lo, hi = node.get("minimum"), node.get("maximum")

        def check_range(v, path, errs, lo=lo, hi=hi):
            if isinstance(v, bool) or not isinstance(v, (int, float)):
                return
            if lo is not None and v < lo:
                errs.append(f"{path}: must be >= {lo}")
            if hi is not None and v > hi:
                errs.append(f"{path}: must be <= {hi}")
        checks.append(check_range)

    if "minLength" in node:
        n = node["minLength"]

        def check_len(v, path, errs, n=n):
            if isinstance(v, str) and len(v) < n:
                errs.append(f"{path}: string shorter than {n}")
        checks.append(check_len)

    if node.get("format") == "date-time":
        def check_dt(v, path, errs):
            if isinstance(v, str) and not _RFC3339.match(v):
                errs.append(f"{path}: does not match format 'date-time'")
        checks.append(check_dt)

    if "items" in node or "minItems" in node:
        item_check = _compile(node["items"]) if "items" in node else None
        min_items = node.get("minItems")

        def check_items(v, path, errs, item_check=item_check, min_items=min_items):
            if not isinstance(v, (list, tuple)):
                return
            if min_items is not None and len(v) < min_items:
                errs.append(f"{path}: array shorter than {min_items}")
            if item_check is not None:
                for i, item in enumerate(v):
                    item_check(item, f"{path}.{i}", errs)
        checks.append(check_items)

    if "properties" in node or "required" in node or "additionalProperties" in node:
        props = {k: _compile(v) for k, v in node.get("properties", {}).items()}
        required = list(node.get("required", ()))
        addl = node.get("additionalProperties", True)
        addl_check: Optional[Checker] = _compile(addl) if isinstance(addl, dict) else None
        forbid = addl is False

        def check_obj(v, path, errs, props=props, required=required, addl_check=addl_check, forbid=forbid):
            if not isinstance(v, dict):
                return
            for key in required:
                if key not in v:
                    errs.append(f"{path or '(root)'}: {key} is required")
            for key, val in v.items():
                sub = f"{path}.{key}" if path else key
                chk = props.get(key)
                if chk is not None:
                    chk(val, sub, errs)
                elif forbid:
                    errs.append(f"{path or '(root)'}: additional property {key} is not allowed")
                elif addl_check is not None:
                    addl_check(val, sub, errs)
        checks.append(check_obj)

    def run(v, path, errs, checks=checks):
        for c in checks:
            c(v, path, errs)
    return run


class CompiledSchema:
    def __init__(self, schema: Dict[str, Any]):
        if not isinstance(schema, dict):
            raise ValueError("schema document must be an object")
        self.schema = schema
        self._check = _compile(schema)

    def errors(self, payload: Any) -> List[str]:
        errs: List[str] = []
        self._check(payload, "", errs)
        return errs

    def validate(self, payload: Any) -> None:
        errs = self.errors(payload)
        if errs:
            raise ValidationError(errs)

    def is_valid(self, payload: Any) -> bool:
        return not self.errors(payload)


_CACHE: Dict[str, CompiledSchema] = {}
_LOCK = threading.Lock()


def compiled(name_or_path: str) -> CompiledSchema:
    """Return a cached compiled schema, by contract name or by a JSON file path."""
    cs = _CACHE.get(name_or_path)
    if cs is not None:
        return cs
    with _LOCK:
        cs = _CACHE.get(name_or_path)
        if cs is None:
            if name_or_path in _schemas.names():
                doc = _schemas.get(name_or_path)
            else:
                with open(name_or_path, "r", encoding="utf-8") as fh:
                    doc = json.load(fh)
            cs = CompiledSchema(doc)
            _CACHE[name_or_path] = cs
    return cs


def to_payload(obj: Any) -> Any:
    if hasattr(obj, "to_dict"):
        return obj.to_dict()
    return obj


def validate(name_or_path: str, payload: Any) -> None:
    """REF ValidateAgainstSchema equivalent (pkg/schema/validator.go:13-41), compiled once."""
    compiled(name_or_path).validate(to_payload(payload))
