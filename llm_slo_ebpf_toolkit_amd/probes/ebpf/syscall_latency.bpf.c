/* syscall_latency_ms: slow read/write system calls (fentry/fexit, no per-call map). */
#include "mislo_probe.h"

char LICENSE[] SEC("license") = "GPL";

struct {
	__uint(type, BPF_MAP_TYPE_HASH);
	__uint(max_entries, 32768);
	__type(key, __u64);
	__type(value, __u64);
} sys_t0 SEC(".maps");

static __always_inline int enter(void)
{
	__u64 key = bpf_get_current_pid_tgid(), now = bpf_ktime_get_ns();
	bpf_map_update_elem(&sys_t0, &key, &now, BPF_ANY);
	return 0;
}

static __always_inline int leave(void)
{
	__u64 key = bpf_get_current_pid_tgid();
	__u64 *t0 = bpf_map_lookup_elem(&sys_t0, &key);
	if (!t0)
		return 0;
	__u64 dt = bpf_ktime_get_ns() - *t0;
	bpf_map_delete_elem(&sys_t0, &key);
	mislo_emit(MISLO_SYSCALL_LATENCY, dt);
	return 0;
}

SEC("fentry/ksys_read")
int BPF_PROG(read_enter) { return enter(); }

SEC("fexit/ksys_read")
int BPF_PROG(read_exit) { return leave(); }

SEC("fentry/ksys_write")
int BPF_PROG(write_enter) { return enter(); }

SEC("fexit/ksys_write")
int BPF_PROG(write_exit) { return leave(); }
