/* Minimal smoke program: per-tgid nanosleep counter in a hash map (no ring traffic);
 * used by `agent --probe-smoke` style checks that the verifier and map creation work. */
#include "vmlinux.h"
#include <bpf/bpf_helpers.h>

char LICENSE[] SEC("license") = "GPL";

struct {
	__uint(type, BPF_MAP_TYPE_HASH);
	__uint(max_entries, 1024);
	__type(key, __u32);
	__type(value, __u64);
} nanosleep_count SEC(".maps");

SEC("tp/syscalls/sys_enter_nanosleep")
int count_nanosleep(void *ctx)
{
	__u32 tgid = bpf_get_current_pid_tgid() >> 32;
	__u64 one = 1, *v = bpf_map_lookup_elem(&nanosleep_count, &tgid);
	if (v)
		__sync_fetch_and_add(v, 1);
	else
		bpf_map_update_elem(&nanosleep_count, &tgid, &one, BPF_NOEXIST);
	return 0;
}
