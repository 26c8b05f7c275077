/* tcp_retransmits_total: a retransmitted segment, valued with its connection's retransmits so
 * far (tcp_sock.total_retrans, already counting this one): the window engine averages a signal's
 * values per incident, so a lossy connection's records climb past REF's "elevated" threshold of
 * 2 retransmits while a one-off retransmit stays at 1.
 *
 * Retransmits mostly run from the retransmit timer (softirq): the current task is whichever one
 * was interrupted, so the record is attributed to the SOCKET's cgroup (the pod that owns the
 * connection) rather than the current task's, and carries no pid; the server address is kept so
 * the record joins the pod's requests on that connection (pod + connection tier). */
#include "mislo_probe.h"

char LICENSE[] SEC("license") = "GPL";

SEC("tp/tcp/tcp_retransmit_skb")
int retransmit(struct trace_event_raw_tcp_event_sk_skb *ctx)
{
	if (ctx->family != 2 /* AF_INET */ && ctx->family != 10 /* AF_INET6 */)
		return 0;
	struct sock *sk = (struct sock *)ctx->skaddr;
	__u32 total = BPF_CORE_READ((struct tcp_sock *)sk, total_retrans);
	__u64 cg = BPF_CORE_READ(sk, sk_cgrp_data.cgroup, kn, id);
	if (mislo_below_floor(MISLO_TCP_RETRANSMIT, total))
		return 0;
	struct mislo_event *e = mislo_reserve_cg(MISLO_TCP_RETRANSMIT, total ? total : 1, 0, 0, cg);
	if (!e)
		return 0;
	e->src_port = ctx->sport;
	e->dst_port = ctx->dport;
	__builtin_memcpy(&e->dst_ip, ctx->daddr, 4);
	mislo_submit(e);
	return 0;
}
