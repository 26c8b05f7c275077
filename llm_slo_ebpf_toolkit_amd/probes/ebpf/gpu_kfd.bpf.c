/* GPU-side kernel signals for MI355X nodes (NEW): complements the rocprofiler-sdk tool
 * (probes/rocprof) for workloads that were not started with it. ROCm compute never reaches the
 * DRM GPU scheduler -- HIP writes AQL packets into KFD user-mode queues and rings their doorbells
 * -- so the hooks are where that path is visible to the kernel and to BPF:
 *
 *   gpu_queue_delay_ms   KFD queue eviction: kprobe kfd_process_evict_queues -> kprobe
 *                        kfd_process_restore_queues, per kfd_process. While evicted (VRAM
 *                        eviction / overcommit, kgd2kfd_quiesce_mm for MMU notifiers and
 *                        userptr invalidation, which call evict) none of the process's queues
 *                        run: the whole span is GPU queue delay of that process, attributed to
 *                        its lead thread's pod (the evicting context is some other task)
 *   rccl_collective_ms   uprobe/uretprobe on librccl's ncclAllReduce / ncclAllGather /
 *                        ncclReduceScatter (host-side enqueue + completion of blocking calls)
 *   hip_activity (map)   uprobes on libamdhip64: kernel launches (hipLaunchKernel,
 *                        hipModuleLaunchKernel, hipExtModuleLaunchKernel, hipGraphLaunch), copies
 *                        (hipMemcpy, hipMemcpyAsync: entry counts, exit times the call), the time
 *                        spent in hipStreamSynchronize / hipDeviceSynchronize /
 *                        hipEventSynchronize; and on libhsa-runtime64 (ROCr) the time its threads
 *                        wait for GPU completion signals (hsa_signal_wait_scacquire /
 *                        hsa_signal_wait_relaxed), per tgid (mislo_gpu_act.h). No ring records:
 *                        the agent's KFD sampler (runtime/csrc/gpusampler.h) reads it to tell a
 *                        pod that is using its GPU from an idle one, and turns the pod's GPU wait
 *                        time into gpu_queue_delay_ms: the share of it other processes' waves held
 *                        that GPU
 *
 * The uprobe programs are attached by the agent to every libamdhip64 / libhsa-runtime64 / librccl
 * the node's processes map (collector/uprobes.py). Records carry the has_gpu flag. */
#include "mislo_probe.h"
#include "mislo_gpu_act.h"

char LICENSE[] SEC("license") = "GPL";

/* amdkfd's process (module BTF: CO-RE relocates the field) */
struct kfd_process {
	struct task_struct *lead_thread;
} __attribute__((preserve_access_index));

struct {
	__uint(type, BPF_MAP_TYPE_LRU_HASH);
	__uint(max_entries, 4096);
	__type(key, __u64);   /* struct kfd_process * */
	__type(value, __u64); /* eviction start */
} kfd_evicted SEC(".maps");

struct {
	__uint(type, BPF_MAP_TYPE_HASH);
	__uint(max_entries, 16384);
	__type(key, __u64);   /* pid_tgid */
	__type(value, __u64); /* call start */
} coll_t0 SEC(".maps");

struct {
	__uint(type, BPF_MAP_TYPE_LRU_HASH);
	__uint(max_entries, 16384);
	__type(key, __u32);   /* host tgid */
	__type(value, struct mislo_hip_act);
} hip_activity SEC(".maps");

struct {
	__uint(type, BPF_MAP_TYPE_LRU_HASH);
	__uint(max_entries, 16384);
	__type(key, __u64);   /* mislo_act_key(pid_tgid, kind) */
	__type(value, __u64); /* call entry */
} act_t0 SEC(".maps");

SEC("kprobe/kfd_process_evict_queues")
int BPF_KPROBE(kfd_evict, struct kfd_process *p)
{
	__u64 key = (__u64)p, now = bpf_ktime_get_ns();
	/* nested evictions (KFD counts them) keep the first start */
	bpf_map_update_elem(&kfd_evicted, &key, &now, BPF_NOEXIST);
	return 0;
}

SEC("kprobe/kfd_process_restore_queues")
int BPF_KPROBE(kfd_restore, struct kfd_process *p)
{
	__u64 key = (__u64)p;
	__u64 *t0 = bpf_map_lookup_elem(&kfd_evicted, &key);
	if (!t0)
		return 0;
	__u64 dt = bpf_ktime_get_ns() - *t0;
	bpf_map_delete_elem(&kfd_evicted, &key);
	if (mislo_below_floor(MISLO_GPU_QUEUE_DELAY, dt))
		return 0;
	struct task_struct *t = BPF_CORE_READ(p, lead_thread);
	if (!t)
		return 0;
	struct mislo_event *e = mislo_reserve_task(MISLO_GPU_QUEUE_DELAY, dt, t);
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

SEC("uprobe")
int BPF_KPROBE(hip_launch)
{
	mislo_act_submit(&hip_activity, bpf_get_current_pid_tgid(), 0, bpf_ktime_get_ns());
	return 0;
}

SEC("uprobe")
int BPF_KPROBE(hip_copy)
{
	__u64 pt = bpf_get_current_pid_tgid(), now = bpf_ktime_get_ns();
	mislo_act_submit(&hip_activity, pt, 1, now);
	mislo_act_enter(&act_t0, pt, MISLO_ACT_COPY, now);
	return 0;
}

SEC("uretprobe")
int BPF_KRETPROBE(hip_copy_exit)
{
	mislo_act_exit(&act_t0, &hip_activity, bpf_get_current_pid_tgid(), MISLO_ACT_COPY, bpf_ktime_get_ns());
	return 0;
}

SEC("uprobe")
int BPF_KPROBE(hip_sync_enter)
{
	mislo_act_enter(&act_t0, bpf_get_current_pid_tgid(), MISLO_ACT_SYNC, bpf_ktime_get_ns());
	return 0;
}

SEC("uretprobe")
int BPF_KRETPROBE(hip_sync_exit)
{
	mislo_act_exit(&act_t0, &hip_activity, bpf_get_current_pid_tgid(), MISLO_ACT_SYNC, bpf_ktime_get_ns());
	return 0;
}

SEC("uprobe")
int BPF_KPROBE(hsa_wait_enter)
{
	mislo_act_enter(&act_t0, bpf_get_current_pid_tgid(), MISLO_ACT_WAIT, bpf_ktime_get_ns());
	return 0;
}

SEC("uretprobe")
int BPF_KRETPROBE(hsa_wait_exit)
{
	mislo_act_exit(&act_t0, &hip_activity, bpf_get_current_pid_tgid(), MISLO_ACT_WAIT, bpf_ktime_get_ns());
	return 0;
}
