/* HIP / ROCr call accounting of gpu_kfd.bpf.c, per host tgid, in one place so the host test
 * (host/gpu_act_host.c) runs exactly the code the uprobes run.
 *
 * A call's entry stores its start under (pid_tgid, kind); its exit adds the call's duration to
 * the process's mislo_hip_act (mislo_record.h):
 *   MISLO_ACT_SYNC  hipStreamSynchronize / hipDeviceSynchronize / hipEventSynchronize
 *   MISLO_ACT_COPY  hipMemcpy / hipMemcpyAsync: copy call latency (hipMemcpy waits for the copy and
 *                   the work queued ahead of it; an async copy blocks when its queue is full)
 *   MISLO_ACT_WAIT  ROCr hsa_signal_wait_scacquire / hsa_signal_wait_relaxed: the runtime's waits
 *                   for a GPU completion signal -- every HIP path that blocks on the device ends in
 *                   one, whichever API the workload calls
 * Nested calls of different kinds (hipMemcpy -> hsa_signal_wait) both count, each in its own
 * field; the same kind re-entered on a thread keeps the outer start (BPF_NOEXIST). The agent's KFD
 * sampler turns a pod's wait time into gpu_queue_delay_ms evidence: the share of it other
 * processes held the GPU (runtime/csrc/gpusampler.cpp). */
#ifndef MISLO_GPU_ACT_H
#define MISLO_GPU_ACT_H

#define MISLO_ACT_SYNC 0u
#define MISLO_ACT_COPY 1u
#define MISLO_ACT_WAIT 2u

/* (pid_tgid, kind) -> start: tgid < 2^22, so bits 60-61 are free for the kind */
static __always_inline __u64 mislo_act_key(__u64 pid_tgid, __u32 kind)
{
	return pid_tgid | ((__u64)(kind & 3u) << 60);
}

static __always_inline struct mislo_hip_act *mislo_act_get(void *act_map, __u32 tgid)
{
	struct mislo_hip_act *a = bpf_map_lookup_elem(act_map, &tgid);
	if (a)
		return a;
	struct mislo_hip_act zero = {};
	bpf_map_update_elem(act_map, &tgid, &zero, BPF_NOEXIST);
	return bpf_map_lookup_elem(act_map, &tgid);
}

static __always_inline void mislo_act_enter(void *t0_map, __u64 pid_tgid, __u32 kind, __u64 now)
{
	__u64 key = mislo_act_key(pid_tgid, kind);
	bpf_map_update_elem(t0_map, &key, &now, BPF_NOEXIST);
}

/* the call's duration (0: no entry seen -- attached mid-call) */
static __always_inline __u64 mislo_act_exit(void *t0_map, void *act_map, __u64 pid_tgid, __u32 kind, __u64 now)
{
	__u64 key = mislo_act_key(pid_tgid, kind);
	__u64 *t0 = bpf_map_lookup_elem(t0_map, &key);
	if (!t0)
		return 0;
	__u64 dt = now > *t0 ? now - *t0 : 0;
	bpf_map_delete_elem(t0_map, &key);
	struct mislo_hip_act *a = mislo_act_get(act_map, (__u32)(pid_tgid >> 32));
	if (!a)
		return dt;
	if (kind == MISLO_ACT_SYNC) {
		__sync_fetch_and_add(&a->sync_ns, dt);
		__sync_fetch_and_add(&a->syncs, 1);
	} else if (kind == MISLO_ACT_COPY) {
		__sync_fetch_and_add(&a->copy_ns, dt);
	} else {
		__sync_fetch_and_add(&a->wait_ns, dt);
		__sync_fetch_and_add(&a->waits, 1);
	}
	return dt;
}

/* a submission (kernel launch or copy) without timing */
static __always_inline void mislo_act_submit(void *act_map, __u64 pid_tgid, int copy, __u64 now)
{
	struct mislo_hip_act *a = mislo_act_get(act_map, (__u32)(pid_tgid >> 32));
	if (!a)
		return;
	if (copy)
		__sync_fetch_and_add(&a->copies, 1);
	else
		__sync_fetch_and_add(&a->launches, 1);
	a->last_ns = now;
}

#endif
