/* tcp_retransmits_total: a retransmitted segment, valued with its connection's retransmits in the
 * current 1-second window (REF counts retransmits per window too: pkg/collector/ringbuf.go:204
 * passes a per-event count, pkg/correlation/retry_storm.go counts per pod within a window). The
 * window engine averages a signal's values per incident, so a lossy connection's records climb
 * past REF's "elevated" threshold of 2 while a one-off retransmit stays at 1 -- and a long-lived
 * keep-alive connection (LLM provider, vector DB) drops back to 1 a second after its loss ended,
 * which the lifetime counter tcp_sock.total_retrans never does.
 *
 * Retransmits mostly run from the retransmit timer (softirq): the current task is whichever one
 * was interrupted, so the record is attributed to the SOCKET's cgroup (the pod that owns the
 * connection) rather than the current task's, and carries no pid; the server address is kept so
 * the record joins the pod's requests on that connection (pod + connection tier). */
#include "mislo_probe.h"

char LICENSE[] SEC("license") = "GPL";

#define RETRANS_WINDOW_NS 1000000000ull

struct retrans_win {
	__u64 start_ns;
	__u64 count;
};

/* per-socket window: LRU, so closed connections age out without a close hook */
struct {
	__uint(type, BPF_MAP_TYPE_LRU_HASH);
	__uint(max_entries, 65536);
	__type(key, __u64); /* struct sock * */
	__type(value, struct retrans_win);
} retrans_windows SEC(".maps");

SEC("tp/tcp/tcp_retransmit_skb")
int retransmit(struct trace_event_raw_tcp_event_sk_skb *ctx)
{
	if (ctx->family != 2 /* AF_INET */ && ctx->family != 10 /* AF_INET6 */)
		return 0;
	struct sock *sk = (struct sock *)ctx->skaddr;
	__u64 key = (__u64)(unsigned long)sk;
	__u64 now = bpf_ktime_get_ns();
	__u64 n = 1;
	struct retrans_win *w = bpf_map_lookup_elem(&retrans_windows, &key);
	if (w && now - w->start_ns < RETRANS_WINDOW_NS) {
		n = __sync_fetch_and_add(&w->count, 1) + 1;
	} else {
		struct retrans_win fresh = {.start_ns = now, .count = 1};
		bpf_map_update_elem(&retrans_windows, &key, &fresh, BPF_ANY);
	}
	__u64 cg = BPF_CORE_READ(sk, sk_cgrp_data.cgroup, kn, id);
	if (mislo_below_floor(MISLO_TCP_RETRANSMIT, n))
		return 0;
	struct mislo_event *e = mislo_reserve_cg(MISLO_TCP_RETRANSMIT, n, 0, 0, cg);
	if (!e)
		return 0;
	e->src_port = ctx->sport;
	e->dst_port = ctx->dport;
	__builtin_memcpy(&e->dst_ip, ctx->daddr, 4);
	mislo_submit(e);
	return 0;
}
