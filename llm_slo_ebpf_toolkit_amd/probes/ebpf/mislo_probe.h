/* Common BPF-side plumbing for the agent's probes (REF ebpf/c/ probes emit through one
 * ring too, REF pkg/collector/ringbuf.go:56-150 drains it).
 *
 * Every probe object shares these maps, pinned by name under /sys/fs/bpf so the agent's
 * loader opens them once:
 *   mislo_events  BPF ring buffer (256 MiB) of 16-byte records: mislo_event16 events and the
 *                 mislo_def16 definitions of newly interned ids (mislo_record.h). The agent
 *                 never copies it: at each window cut it DMAs the framed bytes [consumer_pos,
 *                 producer_pos) from the page-locked mapping straight into GPU memory, where
 *                 the definitions are applied and the events decoded (ops/csrc/decode.hip);
 *   mislo_cfg     array: [0] realtime - monotonic offset (ns), [1] node id,
 *                 [2 + type] per-signal emit floor (raw units; the overhead guard raises
 *                 floors before it detaches probes), [124] current epoch (realtime ns with
 *                 the low 2 bits replaced by the epoch tag; the agent publishes one per window
 *                 cut and ships the last 4 bases with the window), [125] trace id counter,
 *                 [126] context id counter;
 *   mislo_traces  LRU trace hash -> trace id in 1 .. 2^24 - 1 (wrapping). LRU eviction only drops
 *                 traces idle far longer than the 2 s correlation window; a re-seen hash gets a
 *                 fresh id with a fresh definition;
 *   mislo_pods    cgroup id -> pod id (agent-populated from the kubelet / CRI);
 *   mislo_ctxs    (pod, pid, conn32) -> context id in 1 .. 2^23 - 1, assigned on first sight.
 *                 When the counter nears the limit the agent clears the map and the counter
 *                 (collector/bpf.py reset_ctx_ids) and ids are defined afresh;
 *   mislo_scratch per-CPU 64-byte mislo_event the probe fills before mislo_submit() packs it.
 * Interning emits the definition record first and inserts the map entry only once the
 * definition is on the ring: any record that carries the id is written after its definition,
 * so ring order is enough for the GPU to resolve it (no map reads on the agent's window path).
 * A definition the ring drops (full) leaves the id unassigned; the event then carries id 0.
 * The userspace model of exactly this logic is runtime/csrc/probesim.cpp (ProbeSim), which
 * the tests and the replay producer drive.
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
#define MISLO_CFG_EPOCH 124
#define MISLO_CFG_TRACE_NEXT 125
#define MISLO_CFG_CTX_NEXT 126

struct mislo_ctx_key {
	__u32 pod_id, pid, conn32, pad;
};

struct {
	__uint(type, BPF_MAP_TYPE_LRU_HASH);
	__uint(max_entries, 1 << 20);
	__type(key, __u64);
	__type(value, __u32);
	__uint(pinning, LIBBPF_PIN_BY_NAME);
} mislo_traces SEC(".maps");

struct {
	__uint(type, BPF_MAP_TYPE_RINGBUF);
	/* 64 MiB = 2.8M framed 24-byte records: 2.8 s of 1M events/s against 1-s window cuts. The
	 * agent page-locks the data for DMA, so this is also its largest resident mapping. */
	__uint(max_entries, 64 * 1024 * 1024);
	__uint(pinning, LIBBPF_PIN_BY_NAME);
} mislo_events SEC(".maps");

/* Split rings (agent --gpus N): shard s >= 1 has its own ring buffer, so each window worker DMAs
 * only its share of the node's records. MISLO_SHARDS rings in all (compile-time: the ring maps
 * are created when the object loads); a pod's shard is in mislo_shards (agent-written: the
 * worker owning the pod's service), pods not in it use ring 0. */
#ifndef MISLO_SHARDS
#define MISLO_SHARDS 8
#endif
#define MISLO_SHARD_RING(n)                                   \
	struct {                                              \
		__uint(type, BPF_MAP_TYPE_RINGBUF);           \
		__uint(max_entries, 16 * 1024 * 1024);        \
		__uint(pinning, LIBBPF_PIN_BY_NAME);          \
	} mislo_events##n SEC(".maps");
#if MISLO_SHARDS > 1
MISLO_SHARD_RING(1)
#endif
#if MISLO_SHARDS > 2
MISLO_SHARD_RING(2)
#endif
#if MISLO_SHARDS > 3
MISLO_SHARD_RING(3)
#endif
#if MISLO_SHARDS > 4
MISLO_SHARD_RING(4)
MISLO_SHARD_RING(5)
MISLO_SHARD_RING(6)
MISLO_SHARD_RING(7)
#endif

struct {
	__uint(type, BPF_MAP_TYPE_HASH);
	__uint(max_entries, 65536);
	__type(key, __u32);   /* pod id */
	__type(value, __u32); /* shard: the ring of the window worker that owns the pod's service */
	__uint(pinning, LIBBPF_PIN_BY_NAME);
} mislo_shards SEC(".maps");

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

struct {
	__uint(type, BPF_MAP_TYPE_HASH);
	__uint(max_entries, 1 << 20);
	__type(key, struct mislo_ctx_key);
	__type(value, __u32); /* context id, 1 .. 2^23 - 1 (0 = the all-zero context) */
	__uint(pinning, LIBBPF_PIN_BY_NAME);
} mislo_ctxs SEC(".maps");

struct {
	__uint(type, BPF_MAP_TYPE_PERCPU_ARRAY);
	__uint(max_entries, 1);
	__type(key, __u32);
	__type(value, struct mislo_event);
} mislo_scratch SEC(".maps");

static __always_inline __u64 mislo_cfg_get(__u32 idx)
{
	__u64 *v = bpf_map_lookup_elem(&mislo_cfg, &idx);
	return v ? *v : 0;
}

/* True when `value` is below the signal's current emit floor. */
static __always_inline int mislo_below_floor(__u16 type, __u64 value)
{
	/* floors exist for types 0-119; the slots above hold the epoch and the id counters */
	return type < 120 && value < mislo_cfg_get(MISLO_CFG_FLOOR(type));
}

/* Process ids in the pod's own pid namespace. A pod's spans (process.pid) and its rocprofiler
 * records (getpid()) carry the pid the process sees inside its container; the kernel hands the
 * probes host pids. Records are therefore stamped with the thread group's pid in the task's
 * innermost pid namespace (the level its struct pid was allocated at) -- the host pid for a task
 * on the host -- so the pod + pid join tier keys every producer the same way. */
#if defined(__bpf__)
static __always_inline __u32 mislo_ns_tgid(struct task_struct *t)
{
	struct pid *p = BPF_CORE_READ(t, group_leader, thread_pid);
	unsigned int lvl = BPF_CORE_READ(p, level);
	return BPF_CORE_READ(p, numbers[lvl].nr);
}
static __always_inline __u32 mislo_cur_ns_tgid(__u32 tgid)
{
	(void)tgid;
	return mislo_ns_tgid((struct task_struct *)bpf_get_current_task());
}
#else /* host build (probes/ebpf/host): no task structs, pids are taken as given */
static __always_inline __u32 mislo_cur_ns_tgid(__u32 tgid) { return tgid; }
#endif

/* The probe's working record (per-CPU scratch, not ring memory) of a task or socket in cgroup
 * ``cg``: fill, then mislo_submit(). ``tgid`` is already in the pod's pid namespace. */
static __always_inline struct mislo_event *mislo_reserve_cg(__u16 type, __u64 value, __u32 tgid, __u32 tid, __u64 cg)
{
	__u32 zero = 0;
	struct mislo_event *e = bpf_map_lookup_elem(&mislo_scratch, &zero);
	if (!e)
		return 0;
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

/* ... attributed to the current task (its cgroup, its pid in its own namespace; ``tgid`` is the
 * host tgid of bpf_get_current_pid_tgid()) */
static __always_inline struct mislo_event *mislo_reserve(__u16 type, __u64 value, __u32 tgid, __u32 tid)
{
	return mislo_reserve_cg(type, value, mislo_cur_ns_tgid(tgid), tid, bpf_get_current_cgroup_id());
}

#if defined(__bpf__)
/* ... attributed to task ``t``, which need not be the current one (the scheduler probes: at
 * sched_switch the current task is the one leaving the CPU): its cgroup v2 group, its pid */
static __always_inline struct mislo_event *mislo_reserve_task(__u16 type, __u64 value, struct task_struct *t)
{
	return mislo_reserve_cg(type, value, mislo_ns_tgid(t), BPF_CORE_READ(t, pid),
				BPF_CORE_READ(t, cgroups, dfl_cgrp, kn, id));
}
#endif

/* records.py conn_hash_np: splitmix64 of (src port, dst port, dst ip); 0 = no connection */
static __always_inline __u64 mislo_conn_key(const struct mislo_event *e)
{
	if (e->conn_h)
		return e->conn_h;
	if (!e->src_port && !e->dst_port)
		return 0;
	__u64 z = (((__u64)e->src_port << 48) | ((__u64)e->dst_port << 32) | e->dst_ip) + 0x9E3779B97F4A7C15ull;
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
	z ^= z >> 31;
	return z ? z : 1;
}

/* Put a 16-byte record on the ring. No wakeup: the agent reads the ring at its window cuts,
 * never from epoll, so a per-record consumer wakeup would be pure overhead. 0 = written. */
static __always_inline long mislo_out(const void *r, __u32 shard)
{
	switch (shard) {
#if MISLO_SHARDS > 1
	case 1:
		return bpf_ringbuf_output(&mislo_events1, (void *)r, 16, BPF_RB_NO_WAKEUP);
#endif
#if MISLO_SHARDS > 2
	case 2:
		return bpf_ringbuf_output(&mislo_events2, (void *)r, 16, BPF_RB_NO_WAKEUP);
#endif
#if MISLO_SHARDS > 3
	case 3:
		return bpf_ringbuf_output(&mislo_events3, (void *)r, 16, BPF_RB_NO_WAKEUP);
#endif
#if MISLO_SHARDS > 4
	case 4:
		return bpf_ringbuf_output(&mislo_events4, (void *)r, 16, BPF_RB_NO_WAKEUP);
	case 5:
		return bpf_ringbuf_output(&mislo_events5, (void *)r, 16, BPF_RB_NO_WAKEUP);
	case 6:
		return bpf_ringbuf_output(&mislo_events6, (void *)r, 16, BPF_RB_NO_WAKEUP);
	case 7:
		return bpf_ringbuf_output(&mislo_events7, (void *)r, 16, BPF_RB_NO_WAKEUP);
#endif
	default:
		return bpf_ringbuf_output(&mislo_events, (void *)r, 16, BPF_RB_NO_WAKEUP);
	}
}

/* the shard (ring) of a pod's records: 0 unless the agent routed the pod elsewhere */
static __always_inline __u32 mislo_shard(__u32 pod_id)
{
	__u32 *s = pod_id ? bpf_map_lookup_elem(&mislo_shards, &pod_id) : 0;
	return s && *s < MISLO_SHARDS ? *s : 0;
}

/* (pod, pid, connection) -> context id, assigned on first sight from counter [126]: the
 * definition goes on the ring first, then the map entry. Two CPUs racing on a new key both
 * define an id; BPF_NOEXIST lets one win and the other re-reads the winner (the loser's
 * definition names an id nothing uses). An exhausted id space yields 0 until the agent
 * resets the map; the all-zero context is id 0 without a map entry. */
static __always_inline __u32 mislo_ctx_id(__u32 pod_id, __u32 pid, __u32 c32, __u32 shard)
{
	if (!pod_id && !pid && !c32)
		return 0;
	/* keyed per shard: a context is defined on every ring its records go to */
	struct mislo_ctx_key k = {.pod_id = pod_id, .pid = pid, .conn32 = c32, .pad = shard};
	__u32 *id = bpf_map_lookup_elem(&mislo_ctxs, &k);
	if (id)
		return *id;
	__u32 idx = MISLO_CFG_CTX_NEXT;
	__u64 *next = bpf_map_lookup_elem(&mislo_cfg, &idx);
	if (!next)
		return 0;
	__u64 fresh = __sync_fetch_and_add(next, 1) + 1;
	if (fresh >= MISLO_KERNEL_CTX_LIMIT)
		return 0;
	__u32 v = (__u32)fresh;
	struct mislo_def16 d = {.a = c32, .tag_id = MISLO_DEF_CTX | (v << 8), .b = pod_id, .c = pid};
	if (mislo_out(&d, shard))
		return 0; /* ring full: leave the context unnamed */
	if (bpf_map_update_elem(&mislo_ctxs, &k, &v, BPF_NOEXIST) == 0)
		return v;
	id = bpf_map_lookup_elem(&mislo_ctxs, &k);
	return id ? *id : 0;
}

/* trace hash -> trace id in 1 .. 2^24 - 1 (wrapping), definition first like mislo_ctx_id;
 * 0 for untraced events */
static __always_inline __u32 mislo_trace_id(__u64 h, __u32 shard)
{
	if (!h)
		return 0;
	/* keyed per shard too (the shard folded into the hash's top bits): every ring defines the
	 * trace ids its records use */
	__u64 key = h ^ ((__u64)shard << 58);
	__u32 *id = bpf_map_lookup_elem(&mislo_traces, &key);
	if (id)
		return *id;
	__u32 idx = MISLO_CFG_TRACE_NEXT;
	__u64 *next = bpf_map_lookup_elem(&mislo_cfg, &idx);
	if (!next)
		return 0;
	__u32 v = mislo_trace_slot(__sync_fetch_and_add(next, 1));
	struct mislo_def16 d = {.a = v, .tag_id = MISLO_DEF_TRACE, .b = (__u32)h, .c = (__u32)(h >> 32)};
	if (mislo_out(&d, shard))
		return 0;
	if (bpf_map_update_elem(&mislo_traces, &key, &v, BPF_NOEXIST) == 0)
		return v;
	id = bpf_map_lookup_elem(&mislo_traces, &key);
	return id ? *id : 0;
}

/* Pack the working record into the 16-byte ring record (timestamp as an offset from the
 * published epoch, tagged with it) and publish it. */
static __always_inline void mislo_submit(struct mislo_event *e)
{
	struct mislo_event16 r;
	__u32 shard = mislo_shard(e->pod_id);
	__u32 ctx = mislo_ctx_id(e->pod_id, e->pid, mislo_conn32(mislo_conn_key(e)), shard);
	__u32 tid = mislo_trace_id(e->trace_h, shard);
	__u32 eidx = MISLO_CFG_EPOCH;
	__u64 *ep = bpf_map_lookup_elem(&mislo_cfg, &eidx);
	__u64 epoch = ep ? *ep : 0;
	__u64 base = epoch & ~3ull;
	if (e->ts_ns == 0)
		r.ts_off = MISLO_TS_ZERO;
	else if ((__u64)e->ts_ns < base)
		r.ts_off = 0; /* stamped before the epoch it read (clock step): clamp */
	else
		r.ts_off = (__u64)e->ts_ns - base >= MISLO_TS_ZERO ? MISLO_TS_ZERO - 1 : (__u32)((__u64)e->ts_ns - base);
	r.ctx_type = (e->signal_type & 0xFFu) | (ctx << 8);
	r.value_milli = mislo_milli(e->signal_type, e->value);
	r.trace_tag = (tid & MISLO_TRACE_ID_MASK) | ((__u32)(epoch & 3) << MISLO_EPOCH_TAG_SHIFT);
	mislo_out(&r, shard);
}

/* Emit a record attributed to the current task. */
static __always_inline void mislo_emit(__u16 type, __u64 value)
{
	if (mislo_below_floor(type, value))
		return;
	__u64 pt = bpf_get_current_pid_tgid();
	struct mislo_event *e = mislo_reserve(type, value, pt >> 32, (__u32)pt);
	if (e)
		mislo_submit(e);
}

#endif /* MISLO_PROBE_H */
