/* connect_latency_ms + connect_errors_total: tcp_v4/v6_connect entry -> return.
 * A negative return emits a connect error record (type 10) with errno, so the error
 * signal is measured rather than derived in user space. */
#include "mislo_probe.h"

char LICENSE[] SEC("license") = "GPL";

struct conn_start {
	__u64 t0;
	struct sock *sk;
};

struct {
	__uint(type, BPF_MAP_TYPE_HASH);
	__uint(max_entries, 16384);
	__type(key, __u64);
	__type(value, struct conn_start);
} conn_inflight SEC(".maps");

static __always_inline int on_enter(struct sock *sk)
{
	__u64 key = bpf_get_current_pid_tgid();
	struct conn_start c = {.t0 = bpf_ktime_get_ns(), .sk = sk};
	bpf_map_update_elem(&conn_inflight, &key, &c, BPF_ANY);
	return 0;
}

static __always_inline int on_exit(int ret)
{
	__u64 key = bpf_get_current_pid_tgid();
	struct conn_start *c = bpf_map_lookup_elem(&conn_inflight, &key);
	if (!c)
		return 0;
	__u64 dt = bpf_ktime_get_ns() - c->t0;
	struct sock *sk = c->sk;
	__u16 sport = BPF_CORE_READ(sk, __sk_common.skc_num);
	__u16 dport = bpf_ntohs(BPF_CORE_READ(sk, __sk_common.skc_dport));
	__u32 daddr = BPF_CORE_READ(sk, __sk_common.skc_daddr);
	bpf_map_delete_elem(&conn_inflight, &key);
	if (!mislo_below_floor(MISLO_CONNECT_LATENCY, dt)) {
		struct mislo_event *e = mislo_reserve(MISLO_CONNECT_LATENCY, dt, key >> 32, (__u32)key);
		if (e) {
			e->src_port = sport;
			e->dst_port = dport;
			e->dst_ip = daddr;
			e->err = ret < 0 ? -ret : 0;
			mislo_submit(e);
		}
	}
	if (ret < 0 && ret != -115 /* EINPROGRESS: non-blocking connect in flight */) {
		struct mislo_event *e = mislo_reserve(MISLO_CONNECT_ERROR, 1, key >> 32, (__u32)key);
		if (e) {
			e->src_port = sport;
			e->dst_port = dport;
			e->dst_ip = daddr;
			e->err = -ret;
			mislo_submit(e);
		}
	}
	return 0;
}

SEC("kprobe/tcp_v4_connect")
int BPF_KPROBE(connect4_enter, struct sock *sk) { return on_enter(sk); }

SEC("kretprobe/tcp_v4_connect")
int BPF_KRETPROBE(connect4_exit, int ret) { return on_exit(ret); }

SEC("kprobe/tcp_v6_connect")
int BPF_KPROBE(connect6_enter, struct sock *sk) { return on_enter(sk); }

SEC("kretprobe/tcp_v6_connect")
int BPF_KRETPROBE(connect6_exit, int ret) { return on_exit(ret); }
