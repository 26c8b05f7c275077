/* GPU-side kernel signals for MI355X nodes (NEW): complements the rocprofiler-sdk tool
 * (probes/rocprof) for workloads that were not started with it.
 *
 *   gpu_queue_delay_ms   drm GPU scheduler: job queued -> job run on the ring
 *                        (gpu_scheduler:drm_sched_job -> drm_run_job, per fence)
 *   rccl_collective_ms   uprobe/uretprobe on librccl's ncclAllReduce / ncclAllGather /
 *                        ncclReduceScatter (host-side enqueue + completion of blocking
 *                        calls; the agent attaches these pinned programs to every librccl
 *                        the node's processes map, collector/uprobes.py)
 * Records carry the has_gpu flag. */
#include "mislo_probe.h"

char LICENSE[] SEC("license") = "GPL";

struct {
	__uint(type, BPF_MAP_TYPE_LRU_HASH);
	__uint(max_entries, 65536);
	__type(key, __u64);   /* scheduler job pointer */
	__type(value, __u64); /* queued time */
} job_q SEC(".maps");

struct {
	__uint(type, BPF_MAP_TYPE_HASH);
	__uint(max_entries, 16384);
	__type(key, __u64);   /* pid_tgid */
	__type(value, __u64); /* call start */
} coll_t0 SEC(".maps");

SEC("tp/gpu_scheduler/drm_sched_job")
int sched_job(struct trace_event_raw_drm_sched_job *ctx)
{
	__u64 job = (__u64)ctx->sched_job, now = bpf_ktime_get_ns();
	bpf_map_update_elem(&job_q, &job, &now, BPF_ANY);
	return 0;
}

SEC("tp/gpu_scheduler/drm_run_job")
int run_job(struct trace_event_raw_drm_sched_job *ctx)
{
	__u64 job = (__u64)ctx->sched_job;
	__u64 *t0 = bpf_map_lookup_elem(&job_q, &job);
	if (!t0)
		return 0;
	__u64 dt = bpf_ktime_get_ns() - *t0;
	bpf_map_delete_elem(&job_q, &job);
	if (mislo_below_floor(MISLO_GPU_QUEUE_DELAY, dt))
		return 0;
	__u64 pt = bpf_get_current_pid_tgid();
	struct mislo_event *e = mislo_reserve(MISLO_GPU_QUEUE_DELAY, dt, pt >> 32, (__u32)pt);
	if (e) {
		e->flags = MISLO_FLAG_HAS_GPU;
		mislo_submit(e);
	}
	return 0;
}

static __always_inline int coll_enter(void)
{
	__u64 pt = bpf_get_current_pid_tgid(), now = bpf_ktime_get_ns();
	bpf_map_update_elem(&coll_t0, &pt, &now, BPF_ANY);
	return 0;
}

static __always_inline int coll_exit(void)
{
	__u64 pt = bpf_get_current_pid_tgid();
	__u64 *t0 = bpf_map_lookup_elem(&coll_t0, &pt);
	if (!t0)
		return 0;
	__u64 dt = bpf_ktime_get_ns() - *t0;
	bpf_map_delete_elem(&coll_t0, &pt);
	if (mislo_below_floor(MISLO_RCCL_COLLECTIVE, dt))
		return 0;
	struct mislo_event *e = mislo_reserve(MISLO_RCCL_COLLECTIVE, dt, pt >> 32, (__u32)pt);
	if (e) {
		e->flags = MISLO_FLAG_HAS_GPU;
		mislo_submit(e);
	}
	return 0;
}

SEC("uprobe")
int BPF_KPROBE(allreduce_enter) { return coll_enter(); }
SEC("uretprobe")
int BPF_KRETPROBE(allreduce_exit) { return coll_exit(); }
SEC("uprobe")
int BPF_KPROBE(allgather_enter) { return coll_enter(); }
SEC("uretprobe")
int BPF_KRETPROBE(allgather_exit) { return coll_exit(); }
SEC("uprobe")
int BPF_KPROBE(reducescatter_enter) { return coll_enter(); }
SEC("uretprobe")
int BPF_KRETPROBE(reducescatter_exit) { return coll_exit(); }
