import importlib
import sys

from . import TOOLS


def main() -> int:
    if len(sys.argv) < 2 or sys.argv[1] not in TOOLS:
        print("usage: python -m llm_slo_ebpf_toolkit_amd.cli {" + "|".join(TOOLS) + "} [flags]", file=sys.stderr)
        return 2
    mod = importlib.import_module(f"{__package__}.{sys.argv[1]}")
    return mod.main(sys.argv[2:])


if __name__ == "__main__":
    sys.exit(main())
