/* runqueue_delay_ms: wakeup -> actually running on a CPU, per task (BTF tracepoints).
 * Attributed to the task that waited (next: its cgroup and its pid in its own namespace, not
 * the outgoing current task's), emitted only above the floor (default set by the agent to
 * 100 us). */
#include "mislo_probe.h"

char LICENSE[] SEC("license") = "GPL";

struct {
	__uint(type, BPF_MAP_TYPE_HASH);
	__uint(max_entries, 32768);
	__type(key, __u32);   /* tid */
	__type(value, __u64); /* enqueue time */
} runq_enq SEC(".maps");

static __always_inline int enqueue(struct task_struct *p)
{
	__u32 tid = BPF_CORE_READ(p, pid);
	__u64 now = bpf_ktime_get_ns();
	bpf_map_update_elem(&runq_enq, &tid, &now, BPF_ANY);
	return 0;
}

SEC("tp_btf/sched_wakeup")
int BPF_PROG(rq_wakeup, struct task_struct *p) { return enqueue(p); }

SEC("tp_btf/sched_wakeup_new")
int BPF_PROG(rq_wakeup_new, struct task_struct *p) { return enqueue(p); }

SEC("tp_btf/sched_switch")
int BPF_PROG(rq_switch, bool preempt, struct task_struct *prev, struct task_struct *next)
{
	/* a preempted task goes straight back onto the run queue */
	if (BPF_CORE_READ(prev, __state) == 0 /* TASK_RUNNING */)
		enqueue(prev);
	__u32 tid = BPF_CORE_READ(next, pid);
	__u64 *t0 = bpf_map_lookup_elem(&runq_enq, &tid);
	if (!t0)
		return 0;
	__u64 dt = bpf_ktime_get_ns() - *t0;
	bpf_map_delete_elem(&runq_enq, &tid);
	if (mislo_below_floor(MISLO_RUNQUEUE_DELAY, dt))
		return 0;
	/* the waiter's own pod and pid: at sched_switch the current task (and cgroup) is prev's */
	struct mislo_event *e = mislo_reserve_task(MISLO_RUNQUEUE_DELAY, dt, next);
	if (e)
		mislo_submit(e);
	return 0;
}
