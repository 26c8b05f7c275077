/* tcp_retransmits_total: one count per retransmitted segment (tracepoint, no state).
 * Unlike a port-only record, the server address is kept so retransmit storms can be
 * joined on the connection (tier pod+conn) and counted per pod (K6 storm kernel). */
#include "mislo_probe.h"

char LICENSE[] SEC("license") = "GPL";

SEC("tp/tcp/tcp_retransmit_skb")
int retransmit(struct trace_event_raw_tcp_event_sk_skb *ctx)
{
	if (ctx->family != 2 /* AF_INET */ && ctx->family != 10 /* AF_INET6 */)
		return 0;
	__u64 pt = bpf_get_current_pid_tgid();
	struct mislo_event *e = mislo_reserve(MISLO_TCP_RETRANSMIT, 1, pt >> 32, (__u32)pt);
	if (!e)
		return 0;
	e->src_port = ctx->sport;
	e->dst_port = ctx->dport;
	__builtin_memcpy(&e->dst_ip, ctx->daddr, 4);
	mislo_submit(e);
	return 0;
}
