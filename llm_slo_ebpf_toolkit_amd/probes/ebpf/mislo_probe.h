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
 *   mislo_scratch per-CPU 64-byte mislo_event the probe fills before mislo_submit() packs it;
 *   mislo_stages  per-CPU staging batch per ring: slots go on the ring 8 to a record (struct
 *                 mislo_batch, 136 ring bytes) -- when the batch is full, when a definition joins
 *                 it, before a slot of a newer epoch joins it, and at the agent's window cut,
 *                 which runs mislo_flush.bpf.c on every CPU (BPF_PROG_TEST_RUN on that CPU)
 *                 after publishing the new epoch. Unused slots of a flushed batch are pads.
 * Interning puts the definition on the ring first (its batch is flushed at once) and inserts the
 * map entry only then: any record that carries the id, on any CPU, is written after its
 * definition, so ring order is enough for the GPU to resolve it (no map reads on the agent's
 * window path).
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

#if defined(__clang__)
#define MISLO_UNROLL _Pragma("unroll")
#else
#define MISLO_UNROLL
#endif

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

/* A CPU's staging batch for one ring (mislo_stage_put). */
struct mislo_stage {
	__u32 n;     /* slots filled */
	__u32 busy;  /* a program of this CPU is inside mislo_stage_put: one that interrupts it (the
	                cut's flush, an NMI-context probe) leaves the batch alone */
	__u64 epoch; /* the epoch the slots were written in (mislo_cfg[MISLO_CFG_EPOCH]) */
	struct mislo_batch b;
};

struct {
	__uint(type, BPF_MAP_TYPE_PERCPU_ARRAY);
	__uint(max_entries, MISLO_SHARDS);
	__type(key, __u32); /* ring (shard) */
	__type(value, struct mislo_stage);
	__uint(pinning, LIBBPF_PIN_BY_NAME);
} mislo_stages SEC(".maps");

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

/* Put a batch on a ring. No wakeup: the agent reads the ring at its window cuts, never from
 * epoll, so a per-record consumer wakeup would be pure overhead. 0 = written. */
#define MISLO_BATCH_BYTES (16 * MISLO_BATCH_SLOTS)
static __always_inline long mislo_ring_out(void *b, __u32 shard)
{
	switch (shard) {
#if MISLO_SHARDS > 1
	case 1:
		return bpf_ringbuf_output(&mislo_events1, b, MISLO_BATCH_BYTES, BPF_RB_NO_WAKEUP);
#endif
#if MISLO_SHARDS > 2
	case 2:
		return bpf_ringbuf_output(&mislo_events2, b, MISLO_BATCH_BYTES, BPF_RB_NO_WAKEUP);
#endif
#if MISLO_SHARDS > 3
	case 3:
		return bpf_ringbuf_output(&mislo_events3, b, MISLO_BATCH_BYTES, BPF_RB_NO_WAKEUP);
#endif
#if MISLO_SHARDS > 4
	case 4:
		return bpf_ringbuf_output(&mislo_events4, b, MISLO_BATCH_BYTES, BPF_RB_NO_WAKEUP);
	case 5:
		return bpf_ringbuf_output(&mislo_events5, b, MISLO_BATCH_BYTES, BPF_RB_NO_WAKEUP);
	case 6:
		return bpf_ringbuf_output(&mislo_events6, b, MISLO_BATCH_BYTES, BPF_RB_NO_WAKEUP);
	case 7:
		return bpf_ringbuf_output(&mislo_events7, b, MISLO_BATCH_BYTES, BPF_RB_NO_WAKEUP);
#endif
	default:
		return bpf_ringbuf_output(&mislo_events, b, MISLO_BATCH_BYTES, BPF_RB_NO_WAKEUP);
	}
}

static __always_inline void mislo_pad_batch(struct mislo_batch *b)
{
MISLO_UNROLL
	for (int j = 0; j < MISLO_BATCH_SLOTS; ++j) {
		b->slot[j].ts_off = 0;
		b->slot[j].ctx_type = MISLO_DEF_PAD;
		b->slot[j].value_milli = 0;
		b->slot[j].trace_tag = 0;
	}
}

/* The batch goes on its ring (a full ring drops it whole); the stage starts over, all pads. */
static __always_inline long mislo_stage_flush(struct mislo_stage *st, __u32 shard)
{
	long rc = mislo_ring_out(&st->b, shard);
	mislo_pad_batch(&st->b);
	st->n = 0;
	return rc;
}

/* A 16-byte slot into this CPU's batch for `shard` (flush_now: a definition -- its batch goes on
 * the ring before the caller publishes the id in a map). 0 = staged / written. */
static __always_inline long mislo_stage_put(const void *slot, __u32 shard, int flush_now)
{
	__u32 key = shard;
	struct mislo_stage *st = bpf_map_lookup_elem(&mislo_stages, &key);
	if (!st)
		return -1;
	__u64 epoch = mislo_cfg_get(MISLO_CFG_EPOCH);
	if (st->busy) { /* this CPU's batch is mid-update below us: a batch of its own */
		struct mislo_batch one;
		mislo_pad_batch(&one);
		__builtin_memcpy(&one.slot[0], slot, 16);
		return mislo_ring_out(&one, shard);
	}
	st->busy = 1;
	if (st->n && st->epoch != epoch) /* a batch holds one epoch's slots */
		mislo_stage_flush(st, shard);
	__u32 n = st->n & (MISLO_BATCH_SLOTS - 1);
	__builtin_memcpy(&st->b.slot[n], slot, 16);
	st->n = n + 1;
	st->epoch = epoch;
	long rc = 0;
	if (st->n >= MISLO_BATCH_SLOTS || flush_now)
		rc = mislo_stage_flush(st, shard);
	st->busy = 0;
	return rc;
}

/* The window cut's flush of this CPU's batches (mislo_flush.bpf.c, run on each CPU in turn). */
static __always_inline void mislo_flush_cpu(void)
{
MISLO_UNROLL
	for (__u32 s = 0; s < MISLO_SHARDS; ++s) {
		__u32 key = s;
		struct mislo_stage *st = bpf_map_lookup_elem(&mislo_stages, &key);
		if (!st || !st->n || st->busy)
			continue;
		st->busy = 1;
		mislo_stage_flush(st, s);
		st->busy = 0;
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
	if (mislo_stage_put(&d, shard, 1))
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
	if (mislo_stage_put(&d, shard, 1))
		return 0;
	if (bpf_map_update_elem(&mislo_traces, &key, &v, BPF_NOEXIST) == 0)
		return v;
	id = bpf_map_lookup_elem(&mislo_traces, &key);
	return id ? *id : 0;
}

/* Pack the working record into its 16-byte slot (timestamp as an offset from the published
 * epoch, tagged with it) and stage it in this CPU's batch. */
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
	mislo_stage_put(&r, shard, 0);
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
