/* dns_latency_ms: UDP query to :53 -> the reply being returned to the same socket.
 *
 * udp_sendmsg (kprobe) records the send time per (task, socket) when the destination port
 * is 53; udp_recvmsg's *return* (kretprobe) closes the pair, so the value is the time
 * until the answer reached the application (a blocking recvmsg entered before the answer
 * arrived is not mistaken for the answer). Conn tuple = the query's ports / server IP. */
#include "mislo_probe.h"

char LICENSE[] SEC("license") = "GPL";

struct dns_query {
	__u64 t0;
	__u32 daddr;
	__u16 sport;
	__u16 dport;
};

struct {
	__uint(type, BPF_MAP_TYPE_LRU_HASH);
	__uint(max_entries, 16384);
	__type(key, __u64);             /* pid_tgid */
	__type(value, struct dns_query);
} dns_inflight SEC(".maps");

SEC("kprobe/udp_sendmsg")
int BPF_KPROBE(dns_send, struct sock *sk)
{
	__u16 dport = bpf_ntohs(BPF_CORE_READ(sk, __sk_common.skc_dport));
	if (dport != 53)
		return 0;
	struct dns_query q = {
		.t0 = bpf_ktime_get_ns(),
		.daddr = BPF_CORE_READ(sk, __sk_common.skc_daddr),
		.sport = BPF_CORE_READ(sk, __sk_common.skc_num),
		.dport = dport,
	};
	__u64 key = bpf_get_current_pid_tgid();
	bpf_map_update_elem(&dns_inflight, &key, &q, BPF_ANY);
	return 0;
}

SEC("kretprobe/udp_recvmsg")
int BPF_KRETPROBE(dns_recv_ret, int ret)
{
	__u64 key = bpf_get_current_pid_tgid();
	struct dns_query *q = bpf_map_lookup_elem(&dns_inflight, &key);
	if (!q || ret < 0)
		return 0;
	__u64 dt = bpf_ktime_get_ns() - q->t0;
	if (!mislo_below_floor(MISLO_DNS_LATENCY, dt)) {
		struct mislo_event *e = mislo_reserve(MISLO_DNS_LATENCY, dt, key >> 32, (__u32)key);
		if (e) {
			e->src_port = q->sport;
			e->dst_port = q->dport;
			e->dst_ip = q->daddr;
			mislo_submit(e);
		}
	}
	bpf_map_delete_elem(&dns_inflight, &key);
	return 0;
}
