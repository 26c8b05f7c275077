/* mem_reclaim_latency_ms: direct-reclaim stalls (vmscan begin -> end) of the allocating task. */
#include "mislo_probe.h"

char LICENSE[] SEC("license") = "GPL";

struct {
	__uint(type, BPF_MAP_TYPE_HASH);
	__uint(max_entries, 16384);
	__type(key, __u64);
	__type(value, __u64);
} reclaim_t0 SEC(".maps");

SEC("tp/vmscan/mm_vmscan_direct_reclaim_begin")
int reclaim_begin(void *ctx)
{
	__u64 key = bpf_get_current_pid_tgid(), now = bpf_ktime_get_ns();
	bpf_map_update_elem(&reclaim_t0, &key, &now, BPF_ANY);
	return 0;
}

SEC("tp/vmscan/mm_vmscan_direct_reclaim_end")
int reclaim_end(void *ctx)
{
	__u64 key = bpf_get_current_pid_tgid();
	__u64 *t0 = bpf_map_lookup_elem(&reclaim_t0, &key);
	if (!t0)
		return 0;
	__u64 dt = bpf_ktime_get_ns() - *t0;
	bpf_map_delete_elem(&reclaim_t0, &key);
	mislo_emit(MISLO_MEM_RECLAIM, dt);
	return 0;
}
