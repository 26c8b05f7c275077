/* hello_sys_enter_write_total: one count per write(2) from the target comms (the loader
 * fills hello_targets with comm names; an empty map means every task). This is the real
 * kernel path of the agent's hello tracer (REF's is timer-driven in user space). */
#include "mislo_probe.h"

char LICENSE[] SEC("license") = "GPL";

struct comm_key {
	char comm[16];
};

struct {
	__uint(type, BPF_MAP_TYPE_HASH);
	__uint(max_entries, 64);
	__type(key, struct comm_key);
	__type(value, __u8);
} hello_targets SEC(".maps");

struct {
	__uint(type, BPF_MAP_TYPE_ARRAY);
	__uint(max_entries, 1);
	__type(key, __u32);
	__type(value, __u32); /* number of configured targets */
} hello_ntargets SEC(".maps");

SEC("tp/syscalls/sys_enter_write")
int hello_write(void *ctx)
{
	__u32 zero = 0;
	__u32 *n = bpf_map_lookup_elem(&hello_ntargets, &zero);
	if (n && *n) {
		struct comm_key k = {};
		bpf_get_current_comm(&k.comm, sizeof(k.comm));
		if (!bpf_map_lookup_elem(&hello_targets, &k))
			return 0;
	}
	mislo_emit(MISLO_HELLO, 1);
	return 0;
}
