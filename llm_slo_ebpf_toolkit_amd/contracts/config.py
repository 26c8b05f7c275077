"""Toolkit configuration: defaults, YAML loading and normalisation.

Parity: REF pkg/toolkitcfg/config.go:11-170 (``Default``, ``Load``, ``normalize``) with
identical defaults and identical "zero value -> default" rules. NEW adds an optional
``gpu`` block (engine knobs) that REF configs simply omit.
"""

from __future__ import annotations

import copy
from dataclasses import asdict, dataclass, field
from typing import Any, Dict, List

import yaml

from ..signals import catalog

API_VERSION = "toolkit.llm-slo.dev/v1alpha1"
KIND = "ToolkitConfig"


@dataclass
class SamplingConfig:
    events_per_second_limit: int = 10000
    burst_limit: int = 20000


@dataclass
class CorrelationConfig:
    window_ms: int = 2000


@dataclass
class OTLPConfig:
    endpoint: str = "http://otel-collector:4317"


@dataclass
class SafetyConfig:
    max_overhead_pct: float = 5.0


@dataclass
class WebhookConfig:
    enabled: bool = False
    url: str = ""
    secret: str = ""
    format: str = "generic"
    timeout_ms: int = 5000


@dataclass
class CDGateConfig:
    enabled: bool = False
    prometheus_url: str = "http://prometheus:9090"
    ttft_p95_ms: float = 800.0
    error_rate: float = 0.05
    burn_rate: float = 2.0
    fail_open: bool = True


@dataclass
class GPUConfig:
    enabled: bool = True
    window_ms: int = 1000
    max_events_per_window: int = 1 << 20
    world_size: int = 1
    attribution_model: str = "bayes"


@dataclass
class ToolkitConfig:
    apiVersion: str = API_VERSION
    kind: str = KIND
    signal_set: List[str] = field(default_factory=lambda: list(catalog.DEFAULT_CONFIG_SIGNALS))
    sampling: SamplingConfig = field(default_factory=SamplingConfig)
    correlation: CorrelationConfig = field(default_factory=CorrelationConfig)
    otlp: OTLPConfig = field(default_factory=OTLPConfig)
    safety: SafetyConfig = field(default_factory=SafetyConfig)
    webhook: WebhookConfig = field(default_factory=WebhookConfig)
    cdgate: CDGateConfig = field(default_factory=CDGateConfig)
    gpu: GPUConfig = field(default_factory=GPUConfig)

    def to_dict(self) -> Dict[str, Any]:
        return asdict(self)


def default() -> ToolkitConfig:
    return ToolkitConfig()


_SECTIONS = {
    "sampling": SamplingConfig, "correlation": CorrelationConfig, "otlp": OTLPConfig,
    "safety": SafetyConfig, "webhook": WebhookConfig, "cdgate": CDGateConfig, "gpu": GPUConfig,
}


def from_mapping(data: Dict[str, Any]) -> ToolkitConfig:
    """Overlay a parsed YAML mapping onto the defaults (yaml.v3 Unmarshal semantics:
    keys present override, absent keys keep defaults, unknown keys are ignored)."""
    cfg = default()
    if not isinstance(data, dict):
        raise ValueError("config document must be a mapping")
    for key in ("apiVersion", "kind"):
        if key in data and data[key] is not None:
            setattr(cfg, key, str(data[key]))
    if "signal_set" in data and data["signal_set"] is not None:
        cfg.signal_set = [str(s) for s in data["signal_set"]]
    for name, klass in _SECTIONS.items():
        section = data.get(name)
        if not isinstance(section, dict):
            continue
        obj = getattr(cfg, name)
        for fname, fdef in klass.__dataclass_fields__.items():
            if fname in section and section[fname] is not None:
                current = getattr(obj, fname)
                val = section[fname]
                if isinstance(current, bool):
                    val = bool(val)
                elif isinstance(current, int):
                    val = int(val)
                elif isinstance(current, float):
                    val = float(val)
                else:
                    val = str(val)
                setattr(obj, fname, val)
    normalize(cfg)
    return cfg


def load(path: str) -> ToolkitConfig:
    """REF toolkitcfg.Load: read + unmarshal over defaults + normalize. Raises on I/O or parse error."""
    with open(path, "r", encoding="utf-8") as fh:
        data = yaml.safe_load(fh)
    if data is None:
        data = {}
    return from_mapping(data)


def normalize(cfg: ToolkitConfig) -> ToolkitConfig:
    """REF normalize (config.go:125-170): non-positive / empty fields fall back to defaults."""
    d = default()
    if not cfg.signal_set:
        cfg.signal_set = list(d.signal_set)
    if cfg.sampling.events_per_second_limit <= 0:
        cfg.sampling.events_per_second_limit = d.sampling.events_per_second_limit
    if cfg.sampling.burst_limit <= 0:
        cfg.sampling.burst_limit = d.sampling.burst_limit
    if cfg.correlation.window_ms <= 0:
        cfg.correlation.window_ms = d.correlation.window_ms
    if not cfg.otlp.endpoint:
        cfg.otlp.endpoint = d.otlp.endpoint
    if cfg.safety.max_overhead_pct <= 0:
        cfg.safety.max_overhead_pct = d.safety.max_overhead_pct
    if not cfg.webhook.format:
        cfg.webhook.format = d.webhook.format
    if cfg.webhook.timeout_ms <= 0:
        cfg.webhook.timeout_ms = d.webhook.timeout_ms
    if not cfg.cdgate.prometheus_url:
        cfg.cdgate.prometheus_url = d.cdgate.prometheus_url
    if cfg.cdgate.ttft_p95_ms <= 0:
        cfg.cdgate.ttft_p95_ms = d.cdgate.ttft_p95_ms
    if cfg.cdgate.error_rate <= 0:
        cfg.cdgate.error_rate = d.cdgate.error_rate
    if cfg.cdgate.burn_rate <= 0:
        cfg.cdgate.burn_rate = d.cdgate.burn_rate
    if not cfg.apiVersion:
        cfg.apiVersion = d.apiVersion
    if not cfg.kind:
        cfg.kind = d.kind
    if cfg.gpu.window_ms <= 0:
        cfg.gpu.window_ms = d.gpu.window_ms
    if cfg.gpu.max_events_per_window <= 0:
        cfg.gpu.max_events_per_window = d.gpu.max_events_per_window
    if cfg.gpu.world_size < 0:  # 0 = every GPU visible to the agent (agent --gpus 0)
        cfg.gpu.world_size = d.gpu.world_size
    return cfg


def dump_yaml(cfg: ToolkitConfig, include_gpu: bool = True) -> str:
    data = copy.deepcopy(cfg.to_dict())
    if not include_gpu:
        data.pop("gpu", None)
    return yaml.safe_dump(data, sort_keys=False)


def resolve_config_path(argv: List[str], fallback: str) -> str:
    """Pre-scan argv for --config (REF cmd/attributor/main.go:155-166, cmd/sloctl/cdgate.go:117-128)."""
    for i, arg in enumerate(argv):
        arg = arg.strip()
        if arg == "--config" and i + 1 < len(argv):
            return argv[i + 1].strip()
        if arg.startswith("--config="):
            return arg[len("--config="):].strip()
    return fallback
