"""Node agent (DaemonSet process): REF cmd/agent/main.go re-designed around the MI355X
window engine. See ``daemon.Agent``."""
