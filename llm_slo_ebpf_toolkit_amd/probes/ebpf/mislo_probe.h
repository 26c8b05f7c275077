/* Common BPF-side plumbing for the agent's probes.
 *
 * Every probe object shares these maps, pinned by name under /sys/fs/bpf so the agent's
 * loader opens them once:
 *   mislo_events  BPF ring buffer of 16-byte mislo_event16 records (20-byte mislo_event20t
 *                 with -DMISLO_RING_EVENT20T, 24-byte mislo_event24 with -DMISLO_RING_EVENT24,
 *                 32-byte mislo_event32 with -DMISLO_RING_EVENT32) that the agent drains into
 *                 the GPU window ring (16 MiB);
 *   mislo_cfg     array: [0] realtime - monotonic offset (ns), [1] node id,
 *                 [2 + type] per-signal emit floor (raw units; the overhead guard raises
 *                 floors before it detaches probes), [124] current epoch (event16 rings:
 *                 realtime ns with the low 2 bits replaced by the epoch tag; the agent
 *                 publishes one per window cut and keeps the last 4 bases), [125] trace id counter,
 *                 [126] context id counter, [127] connection id counter;
 *   mislo_traces  LRU trace hash -> 32-bit trace id (event20t rings). Trace ids are per request
 *                 and never reused within 2^32 - 1 assignments; LRU eviction only drops traces
 *                 idle for far longer than the 2 s correlation window. The agent looks up the
 *                 window's span trace hashes here (spans of traces no probe saw get ids from
 *                 a disjoint range and match nothing, as they should);
 *   mislo_pods    cgroup id -> pod id (agent-populated from the kubelet / CRI);
 *   mislo_conns   connection key -> 24-bit connection id, assigned here on first sight; the
 *                 agent reads it (batch lookup, per window) to put spans on the same ids;
 *   mislo_ctxs    (pod, pid, connection id) -> 24-bit context id, assigned here on first
 *                 sight. When counter [126] has moved since the last window, the agent
 *                 batch-reads the map after snapshotting the ring (every id a snapshotted
 *                 record carries was inserted before the record was written) and appends
 *                 the new rows (pod, pid, conn, svc|node from pod metadata) to the device
 *                 context table before the window's DMA;
 *   mislo_scratch per-CPU 64-byte mislo_event the probe fills before mislo_submit() packs it.
 * Records are stamped with wall-clock ns, their connections interned and their values
 * converted to fixed point in the kernel, so the consumer copies ring bytes straight into
 * pinned memory and DMAs them to the GPU without touching individual records.
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
#define MISLO_CFG_CONN_NEXT 127
#define MISLO_CONN_ID_LIMIT (1u << 24)

struct mislo_ctx_key {
	__u32 pod_id, pid, conn_id, pad;
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

struct {
	__uint(type, BPF_MAP_TYPE_HASH);
	__uint(max_entries, 1 << 20);
	__type(key, __u64);   /* connection key (records.py conn keys) */
	__type(value, __u32); /* connection id, 1 .. 2^24 - 1 */
	__uint(pinning, LIBBPF_PIN_BY_NAME);
} mislo_conns SEC(".maps");

struct {
	__uint(type, BPF_MAP_TYPE_HASH);
	__uint(max_entries, 1 << 20);
	__type(key, struct mislo_ctx_key);
	__type(value, __u32); /* context id, 1 .. 2^24 - 1 (0 = the all-zero context) */
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
	return value < mislo_cfg_get(MISLO_CFG_FLOOR(type));
}

/* The probe's working record (per-CPU scratch, not ring memory): fill, then mislo_submit(). */
static __always_inline struct mislo_event *mislo_reserve(__u16 type, __u64 value, __u32 tgid, __u32 tid)
{
	__u32 zero = 0;
	struct mislo_event *e = bpf_map_lookup_elem(&mislo_scratch, &zero);
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

/* key -> id from map `m`, assigned on first sight from counter cfg[`ctr`]. Two CPUs racing on
 * a new key both draw ids; BPF_NOEXIST lets one win and the other re-reads the winner (the
 * loser's id is never used). An exhausted id space yields 0 until the agent resets the map. */
#define MISLO_INTERN(m, keyp, ctr)                                                         \
	({                                                                                  \
		__u32 _r = 0;                                                               \
		__u32 *_id = bpf_map_lookup_elem(&(m), (keyp));                             \
		if (_id) {                                                                  \
			_r = *_id;                                                          \
		} else {                                                                    \
			__u32 _idx = (ctr);                                                 \
			__u64 *_next = bpf_map_lookup_elem(&mislo_cfg, &_idx);              \
			if (_next) {                                                        \
				__u64 _fresh = __sync_fetch_and_add(_next, 1) + 1;          \
				if (_fresh < MISLO_CONN_ID_LIMIT) {                         \
					__u32 _v = (__u32)_fresh;                           \
					if (bpf_map_update_elem(&(m), (keyp), &_v, BPF_NOEXIST) == 0) \
						_r = _v;                                    \
					else if ((_id = bpf_map_lookup_elem(&(m), (keyp))))  \
						_r = *_id;                                  \
				}                                                           \
			}                                                                   \
		}                                                                           \
		_r;                                                                         \
	})

static __always_inline __u32 mislo_conn_id(__u64 key)
{
	if (!key)
		return 0;
	return MISLO_INTERN(mislo_conns, &key, MISLO_CFG_CONN_NEXT);
}

/* (pod, pid, connection) -> context id; the all-zero context is id 0 without a map entry */
static __always_inline __u32 mislo_ctx_id(__u32 pod_id, __u32 pid, __u32 conn_id)
{
	if (!pod_id && !pid && !conn_id)
		return 0;
	struct mislo_ctx_key k = {.pod_id = pod_id, .pid = pid, .conn_id = conn_id, .pad = 0};
	return MISLO_INTERN(mislo_ctxs, &k, MISLO_CFG_CTX_NEXT);
}

/* trace hash -> 32-bit id in [1, 2^32 - 1] (wrapping), assigned on first sight like
 * MISLO_INTERN; 0 for untraced events */
static __always_inline __u32 mislo_trace_id(__u64 h)
{
	if (!h)
		return 0;
	__u32 *id = bpf_map_lookup_elem(&mislo_traces, &h);
	if (id)
		return *id;
	__u32 idx = MISLO_CFG_TRACE_NEXT;
	__u64 *next = bpf_map_lookup_elem(&mislo_cfg, &idx);
	if (!next)
		return 0;
	__u64 fresh = __sync_fetch_and_add(next, 1);
	__u32 v = (__u32)(fresh % MISLO_TRACE_ID_MASK) + 1; /* [1, 2^30 - 1]: event16 keeps 2 tag bits */
	if (bpf_map_update_elem(&mislo_traces, &h, &v, BPF_NOEXIST) == 0)
		return v;
	id = bpf_map_lookup_elem(&mislo_traces, &h);
	return id ? *id : 0;
}

/* Pack the working record into the ring record and publish it. */
static __always_inline void mislo_submit(struct mislo_event *e)
{
	__u32 cid = mislo_conn_id(mislo_conn_key(e));
#ifdef MISLO_RING_EVENT32
	struct mislo_event32 r;
	r.ts_ns = e->ts_ns;
	r.trace_h = e->trace_h;
	r.value_milli = mislo_milli(e->signal_type, e->value);
	r.pid = e->pid;
	r.pod_id = e->pod_id;
	r.type_conn = (e->signal_type & 0xFFu) | (cid << 8);
#elif defined(MISLO_RING_EVENT20T)
	struct mislo_event20t r;
	r.ts_ns = e->ts_ns;
	r.value_milli = mislo_milli(e->signal_type, e->value);
	r.ctx_type = (e->signal_type & 0xFFu) | (mislo_ctx_id(e->pod_id, e->pid, cid) << 8);
	r.trace_id = mislo_trace_id(e->trace_h);
#elif defined(MISLO_RING_EVENT24)
	struct mislo_event24 r;
	r.ts_ns = e->ts_ns;
	r.trace_h = e->trace_h;
	r.value_milli = mislo_milli(e->signal_type, e->value);
	r.ctx_type = (e->signal_type & 0xFFu) | (mislo_ctx_id(e->pod_id, e->pid, cid) << 8);
#else
	/* default: 16-byte record, timestamp offset from the published epoch, tagged with it */
	struct mislo_event16 r;
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
	r.ctx_type = (e->signal_type & 0xFFu) | (mislo_ctx_id(e->pod_id, e->pid, cid) << 8);
	r.value_milli = mislo_milli(e->signal_type, e->value);
	r.trace_tag = (mislo_trace_id(e->trace_h) & MISLO_TRACE_ID_MASK) | ((__u32)(epoch & 3) << MISLO_EPOCH_TAG_SHIFT);
#endif
	bpf_ringbuf_output(&mislo_events, &r, sizeof(r), 0);
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
