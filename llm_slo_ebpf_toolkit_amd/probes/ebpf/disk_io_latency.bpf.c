/* disk_io_latency_ms: block request issue -> completion keyed by (dev, sector). The
 * completion runs in interrupt / other-task context, so the record is attributed to the
 * task that issued the request (remembered at issue), not to whoever completes it. */
#include "mislo_probe.h"

char LICENSE[] SEC("license") = "GPL";

struct rq_key {
	__u32 dev;
	__u32 pad;
	__u64 sector;
};

struct rq_val {
	__u64 t0;
	__u64 pid_tgid;
};

struct {
	__uint(type, BPF_MAP_TYPE_HASH);
	__uint(max_entries, 32768);
	__type(key, struct rq_key);
	__type(value, struct rq_val);
} rq_start SEC(".maps");

SEC("tp/block/block_rq_issue")
int rq_issue(struct trace_event_raw_block_rq *ctx)
{
	struct rq_key k = {.dev = ctx->dev, .sector = ctx->sector};
	struct rq_val v = {.t0 = bpf_ktime_get_ns(), .pid_tgid = bpf_get_current_pid_tgid()};
	bpf_map_update_elem(&rq_start, &k, &v, BPF_ANY);
	return 0;
}

SEC("tp/block/block_rq_complete")
int rq_complete(struct trace_event_raw_block_rq_completion *ctx)
{
	struct rq_key k = {.dev = ctx->dev, .sector = ctx->sector};
	struct rq_val *v = bpf_map_lookup_elem(&rq_start, &k);
	if (!v)
		return 0;
	__u64 dt = bpf_ktime_get_ns() - v->t0;
	__u64 pt = v->pid_tgid;
	bpf_map_delete_elem(&rq_start, &k);
	if (mislo_below_floor(MISLO_DISK_IO_LATENCY, dt))
		return 0;
	struct mislo_event *e = mislo_reserve(MISLO_DISK_IO_LATENCY, dt, pt >> 32, (__u32)pt);
	if (e)
		mislo_submit(e);
	return 0;
}
