/* The agent's window cut for batched rings: after publishing the new epoch in mislo_cfg, the
 * agent runs this program once on every CPU (BPF_PROG_TEST_RUN with BPF_F_TEST_RUN_ON_CPU,
 * collector/bpf.py BpfMaps.flush_cpus), so each CPU's partially filled staging batches
 * (mislo_probe.h mislo_stages) go on the rings before the agent snapshots their producer
 * positions: no staged slot waits past the cut that follows it. Loaded without attachment
 * (bpftool prog load ... pinmaps: it shares the pinned maps of the probes). */
#include "mislo_probe.h"

char LICENSE[] SEC("license") = "GPL";

SEC("raw_tp")
int mislo_flush(void *ctx)
{
	(void)ctx;
	mislo_flush_cpu();
	return 0;
}
