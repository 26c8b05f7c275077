/* tls_handshake_ms + tls_handshake_fail_total: uprobes on the workloads' libssl
 * SSL_do_handshake. The sections name no binary: the loader pins these programs and the agent
 * attaches them to every libssl the node's processes map, resolved through /proc/<pid>/maps
 * (collector/uprobes.py: ELF symbol offset, perf_event_open + BPF_LINK_CREATE). Non-blocking handshakes return -1 with
 * WANT_READ/WANT_WRITE several times; the handshake time runs from the first call to the
 * call that returns 1, and a final failure (ret <= 0 after which the SSL* is not retried
 * within the window) is counted by the agent from the ret == 0 case reported here. */
#include "mislo_probe.h"

char LICENSE[] SEC("license") = "GPL";

struct {
	__uint(type, BPF_MAP_TYPE_LRU_HASH);
	__uint(max_entries, 16384);
	__type(key, __u64);   /* SSL* */
	__type(value, __u64); /* first-call time */
} tls_start SEC(".maps");

struct {
	__uint(type, BPF_MAP_TYPE_HASH);
	__uint(max_entries, 16384);
	__type(key, __u64);   /* pid_tgid */
	__type(value, __u64); /* SSL* of the call in flight */
} tls_call SEC(".maps");

SEC("uprobe")
int BPF_KPROBE(tls_enter, void *ssl)
{
	__u64 s = (__u64)ssl, now = bpf_ktime_get_ns(), pt = bpf_get_current_pid_tgid();
	bpf_map_update_elem(&tls_start, &s, &now, BPF_NOEXIST);  /* keep the first attempt */
	bpf_map_update_elem(&tls_call, &pt, &s, BPF_ANY);
	return 0;
}

SEC("uretprobe")
int BPF_KRETPROBE(tls_exit, int ret)
{
	__u64 pt = bpf_get_current_pid_tgid();
	__u64 *s = bpf_map_lookup_elem(&tls_call, &pt);
	if (!s)
		return 0;
	__u64 ssl = *s;
	bpf_map_delete_elem(&tls_call, &pt);
	if (ret < 0)
		return 0;  /* WANT_READ / WANT_WRITE: handshake still in progress */
	__u64 *t0 = bpf_map_lookup_elem(&tls_start, &ssl);
	if (!t0)
		return 0;
	__u64 dt = bpf_ktime_get_ns() - *t0;
	bpf_map_delete_elem(&tls_start, &ssl);
	if (ret == 1) {
		if (!mislo_below_floor(MISLO_TLS_HANDSHAKE, dt)) {
			struct mislo_event *e = mislo_reserve(MISLO_TLS_HANDSHAKE, dt, pt >> 32, (__u32)pt);
			if (e) {
				e->dst_port = 443;
				mislo_submit(e);
			}
		}
	} else {
		struct mislo_event *e = mislo_reserve(MISLO_TLS_FAIL, 1, pt >> 32, (__u32)pt);
		if (e) {
			e->dst_port = 443;
			e->err = 1;
			mislo_submit(e);
		}
	}
	return 0;
}
