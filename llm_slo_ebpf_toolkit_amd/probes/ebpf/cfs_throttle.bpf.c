/* cfs_throttled_ms (NEW; REF only synthesises it): time a cgroup's CFS run queue spends
 * throttled by its CPU quota, throttle_cfs_rq -> unthrottle_cfs_rq, attributed to the
 * throttled cgroup's pod. */
#include "mislo_probe.h"

char LICENSE[] SEC("license") = "GPL";

struct {
	__uint(type, BPF_MAP_TYPE_HASH);
	__uint(max_entries, 16384);
	__type(key, __u64);   /* cfs_rq pointer */
	__type(value, __u64); /* throttle time */
} throttled SEC(".maps");

SEC("kprobe/throttle_cfs_rq")
int BPF_KPROBE(cfs_throttle, void *cfs_rq)
{
	__u64 k = (__u64)cfs_rq, now = bpf_ktime_get_ns();
	bpf_map_update_elem(&throttled, &k, &now, BPF_ANY);
	return 0;
}

SEC("kprobe/unthrottle_cfs_rq")
int BPF_KPROBE(cfs_unthrottle, void *cfs_rq)
{
	__u64 k = (__u64)cfs_rq;
	__u64 *t0 = bpf_map_lookup_elem(&throttled, &k);
	if (!t0)
		return 0;
	__u64 dt = bpf_ktime_get_ns() - *t0;
	bpf_map_delete_elem(&throttled, &k);
	mislo_emit(MISLO_CFS_THROTTLE, dt);
	return 0;
}
