/* cpu_steal_pct: share of wall time a task spent runnable-but-waiting, per CPU, reported
 * as milli-percent once per >= 100 ms accounting period (sched_stat_wait delivers each
 * wait interval; summing them per CPU gives the steal-like contention ratio the Bayes
 * model thresholds at 2 % / 8 %). */
#include "mislo_probe.h"

char LICENSE[] SEC("license") = "GPL";

#define STEAL_PERIOD_NS (100ull * 1000 * 1000)

struct steal_acc {
	__u64 period_start;
	__u64 waited;
};

struct {
	__uint(type, BPF_MAP_TYPE_PERCPU_ARRAY);
	__uint(max_entries, 1);
	__type(key, __u32);
	__type(value, struct steal_acc);
} steal_acc SEC(".maps");

SEC("tp/sched/sched_stat_wait")
int stat_wait(struct trace_event_raw_sched_stat_runtime *ctx)
{
	__u32 zero = 0;
	struct steal_acc *a = bpf_map_lookup_elem(&steal_acc, &zero);
	if (!a)
		return 0;
	__u64 now = bpf_ktime_get_ns();
	if (!a->period_start)
		a->period_start = now;
	a->waited += ctx->runtime;  /* the wait interval (ns) */
	__u64 span = now - a->period_start;
	if (span < STEAL_PERIOD_NS)
		return 0;
	__u64 milli_pct = a->waited * 100000ull / span;
	a->period_start = now;
	a->waited = 0;
	mislo_emit(MISLO_CPU_STEAL, milli_pct);
	return 0;
}
