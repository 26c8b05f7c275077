/* Common BPF-side plumbing for the agent's probes.
 *
 * Every probe object shares three maps, pinned by name under /sys/fs/bpf so the agent's
 * loader opens them once:
 *   mislo_events  BPF ring buffer the agent drains into the GPU window ring (16 MiB);
 *   mislo_cfg     array: [0] realtime - monotonic offset (ns), [1] node id,
 *                 [2 + type] per-signal emit floor (raw units; the overhead guard raises
 *                 floors before it detaches probes);
 *   mislo_pods    cgroup id -> pod id (agent-populated from the kubelet / CRI).
 * Records are stamped with wall-clock ns in the kernel, so the consumer copies ring bytes
 * straight into pinned memory without touching individual records.
 */
#ifndef MISLO_PROBE_H
#define MISLO_PROBE_H

#include "vmlinux.h"
#include <bpf/bpf_core_read.h>
#include <bpf/bpf_endian.h>
#include <bpf/bpf_helpers.h>
#include <bpf/bpf_tracing.h>

#include "mislo_record.h"

#define MISLO_CFG_CLOCK 0
#define MISLO_CFG_NODE 1
#define MISLO_CFG_FLOOR(t) (2 + (t))
#define MISLO_CFG_SLOTS 128

struct {
	__uint(type, BPF_MAP_TYPE_RINGBUF);
	__uint(max_entries, 16 * 1024 * 1024);
	__uint(pinning, LIBBPF_PIN_BY_NAME);
} mislo_events SEC(".maps");

struct {
	__uint(type, BPF_MAP_TYPE_ARRAY);
	__uint(max_entries, MISLO_CFG_SLOTS);
	__type(key, __u32);
	__type(value, __u64);
	__uint(pinning, LIBBPF_PIN_BY_NAME);
} mislo_cfg SEC(".maps");

struct {
	__uint(type, BPF_MAP_TYPE_HASH);
	__uint(max_entries, 65536);
	__type(key, __u64);   /* cgroup id */
	__type(value, __u32); /* pod id */
	__uint(pinning, LIBBPF_PIN_BY_NAME);
} mislo_pods SEC(".maps");

static __always_inline __u64 mislo_cfg_get(__u32 idx)
{
	__u64 *v = bpf_map_lookup_elem(&mislo_cfg, &idx);
	return v ? *v : 0;
}

/* True when `value` is below the signal's current emit floor. */
static __always_inline int mislo_below_floor(__u16 type, __u64 value)
{
	return value < mislo_cfg_get(MISLO_CFG_FLOOR(type));
}

static __always_inline struct mislo_event *mislo_reserve(__u16 type, __u64 value, __u32 tgid, __u32 tid)
{
	struct mislo_event *e = bpf_ringbuf_reserve(&mislo_events, sizeof(*e), 0);
	if (!e)
		return 0;
	__u64 cg = bpf_get_current_cgroup_id();
	__u32 *pod = bpf_map_lookup_elem(&mislo_pods, &cg);
	e->ts_ns = (__s64)(bpf_ktime_get_ns() + mislo_cfg_get(MISLO_CFG_CLOCK));
	e->value = value;
	e->trace_h = 0;
	e->pid = tgid;
	e->tid = tid;
	e->pod_id = pod ? *pod : 0;
	e->dst_ip = 0;
	e->signal_type = type;
	e->node_id = (__u16)mislo_cfg_get(MISLO_CFG_NODE);
	e->svc_id = 0;
	e->flags = 0;
	e->src_port = 0;
	e->dst_port = 0;
	e->err = 0;
	e->conn_h = 0;
	return e;
}

/* Emit a record attributed to the current task. */
static __always_inline void mislo_emit(__u16 type, __u64 value)
{
	if (mislo_below_floor(type, value))
		return;
	__u64 pt = bpf_get_current_pid_tgid();
	struct mislo_event *e = mislo_reserve(type, value, pt >> 32, (__u32)pt);
	if (e)
		bpf_ringbuf_submit(e, 0);
}

#endif /* MISLO_PROBE_H */
