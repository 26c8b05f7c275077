"""Command-line tools with REF's binary names and flag surfaces.

Run as ``python -m llm_slo_ebpf_toolkit_amd.cli <tool> [flags]`` or through the
``bin/<tool>`` wrappers: agent, collector, attributor, benchgen, faultreplay, faultinject,
correlationeval, m5gate, sloctl, loadgen, schemavalidate.
"""

TOOLS = ("agent", "collector", "attributor", "benchgen", "faultreplay", "faultinject", "correlationeval", "m5gate",
         "sloctl", "loadgen", "schemavalidate")
