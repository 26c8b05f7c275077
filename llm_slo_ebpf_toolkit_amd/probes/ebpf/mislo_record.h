/* Event records shared by the probes, the rocprofiler tool, the native ring and the GPU
 * decode kernels. Only fixed-width types, so it compiles for the BPF target and for the host
 * layout test.
 *   struct mislo_event   (64 B, collector/records.py EVENT): the probes' working record (per-CPU
 *                        scratch) and the user-space producers' ring record (rocprofiler tool);
 *   struct mislo_event16 (16 B, records.py EVENT16): the slot the probes put on the BPF ring,
 *                        8 to a ring record (struct mislo_batch). The timestamp is a 32-bit offset from the epoch the agent last
 *                        published (mislo_cfg[MISLO_CFG_EPOCH]) and that epoch's 2-bit tag sits
 *                        in the top of trace_tag, so records written across a window cut decode
 *                        exactly (a window carries its last 4 epoch bases). The value is fixed
 *                        point (mislo_milli); the (pod, pid, connection) context and the trace
 *                        hash are interned in the kernel (mislo_probe.h), so the agent DMAs the
 *                        ring bytes to the GPU without reading a record;
 *   definition records   (16 B, same stride, signal-type byte >= MISLO_DEF_FIRST): an interned
 *                        id's meaning, committed to the ring BEFORE the id enters its map, so in
 *                        ring order every definition precedes any record that uses the id:
 *                          MISLO_DEF_CTX   {conn32, 0xFE | ctx id << 8, pod id, pid}
 *                          MISLO_DEF_TRACE {trace id, 0xFD, trace hash lo, trace hash hi}
 *                        The GPU applies them to its context table / trace map in ring order
 *                        (ops/csrc/decode.hip k_ring_defs). */
#ifndef MISLO_RECORD_H
#define MISLO_RECORD_H

#include <linux/types.h>

#ifndef __always_inline
#define __always_inline inline __attribute__((always_inline))
#endif

enum mislo_signal_type {
	MISLO_DNS_LATENCY = 1,      /* ns */
	MISLO_TCP_RETRANSMIT = 2,   /* count */
	MISLO_RUNQUEUE_DELAY = 3,   /* ns */
	MISLO_CONNECT_LATENCY = 4,  /* ns */
	MISLO_TLS_HANDSHAKE = 5,    /* ns */
	MISLO_CPU_STEAL = 6,        /* milli-percent */
	MISLO_MEM_RECLAIM = 7,      /* ns */
	MISLO_DISK_IO_LATENCY = 8,  /* ns */
	MISLO_SYSCALL_LATENCY = 9,  /* ns */
	MISLO_CONNECT_ERROR = 10,   /* count */
	MISLO_TLS_FAIL = 11,        /* count */
	MISLO_CFS_THROTTLE = 12,    /* ns */
	MISLO_GPU_QUEUE_DELAY = 13, /* ns */
	MISLO_HBM_PRESSURE = 14,    /* milli-percent */
	MISLO_XGMI_LATENCY = 15,    /* ns */
	MISLO_RCCL_COLLECTIVE = 16, /* ns */
	MISLO_HELLO = 100,          /* count */
	MISLO_NANOSLEEP = 101,      /* count (minimal probe) */
};

#define MISLO_FLAG_HAS_GPU (1u << 8)

struct mislo_event {
	__s64 ts_ns;       /* CLOCK_REALTIME ns (stamped in-kernel via the agent's offset) */
	__u64 value;       /* raw value in the signal's kernel unit */
	__u64 trace_h;     /* trace-id hash (0 = none; set by user-space producers) */
	__u32 pid;         /* tgid */
	__u32 tid;
	__u32 pod_id;      /* cgroup -> pod id (agent-populated map), 0 = unknown */
	__u32 dst_ip;      /* IPv4 as read from the socket */
	__u16 signal_type;
	__u16 node_id;
	__u16 svc_id;
	__u16 flags;       /* bits 0-7 gpu id, bit 8 has_gpu */
	__u16 src_port;
	__u16 dst_port;
	__s32 err;
	__u64 conn_h;      /* 0: derived on the GPU from (ports, ip) */
};

#define MISLO_EPOCH_TAG_SHIFT 30
#define MISLO_TRACE_ID_MASK ((1u << MISLO_EPOCH_TAG_SHIFT) - 1u)
#define MISLO_TS_ZERO 0xFFFFFFFFu

struct mislo_event16 {
	__u32 ts_off;      /* ns since the tagged epoch; MISLO_TS_ZERO = no timestamp */
	__u32 ctx_type;    /* bits 0-7 signal type, bits 8-31 interned context id (0 = none) */
	__u32 value_milli; /* value in 1/1000 of the signal's output unit (mislo_milli) */
	__u32 trace_tag;   /* bits 0-29 interned trace id (0 = none), bits 30-31 epoch tag */
};

/* definition slots (same 16 bytes as mislo_event16) */
#define MISLO_DEF_FIRST 0xF0u
#define MISLO_DEF_PAD 0xFCu   /* an unused slot of a batch flushed before it filled: {0, 0xFC, 0, 0} */
#define MISLO_DEF_TRACE 0xFDu
#define MISLO_DEF_CTX 0xFEu

/* The ring record: a batch of 16-byte slots a CPU staged (mislo_probe.h mislo_stage_put), one
 * 8-byte ring header per MISLO_BATCH_SLOTS slots -- 17 ring bytes per event instead of 24. */
#define MISLO_BATCH_SLOTS 8
struct mislo_batch {
	struct mislo_event16 slot[MISLO_BATCH_SLOTS];
};
struct mislo_def16 {
	__u32 a;       /* ctx: conn32; trace: trace id */
	__u32 tag_id;  /* bits 0-7 MISLO_DEF_*, bits 8-31 ctx id (ctx definitions) */
	__u32 b;       /* ctx: pod id; trace: hash bits 0-31 */
	__u32 c;       /* ctx: pid; trace: hash bits 32-63 */
};

/* gpu_kfd.bpf.c hip_activity value, per host tgid: the HIP runtime calls of a process (uprobes on
 * libamdhip64), read by the agent's KFD sampler (runtime/csrc/gpusampler.h HipActivity) */
struct mislo_hip_act {
	__u64 launches;   /* hipLaunchKernel / hipModuleLaunchKernel / hipExtModuleLaunchKernel / hipGraphLaunch */
	__u64 copies;     /* hipMemcpy / hipMemcpyAsync calls */
	__u64 last_ns;    /* bpf_ktime of the latest submission */
	__u64 sync_ns;    /* total time in hipStreamSynchronize / hipDeviceSynchronize / hipEventSynchronize */
	__u64 syncs;
	__u64 copy_ns;    /* total time in hipMemcpy / hipMemcpyAsync calls (mislo_gpu_act.h) */
	__u64 wait_ns;    /* total time in ROCr hsa_signal_wait_scacquire / hsa_signal_wait_relaxed */
	__u64 waits;
};

/* id spaces: the kernel assigns the low part, the agent's host-side encoders the rest, so both
 * kinds of producer share one device context table (2^24 rows) and one trace-id space */
#define MISLO_KERNEL_CTX_LIMIT (1u << 23)   /* kernel context ids 1 .. 2^23 - 1 */
#define MISLO_KERNEL_TRACE_LIMIT (1u << 24) /* kernel trace ids 1 .. 2^24 - 1 (mislo_traces holds 2^20) */

/* records.py conn32: the 32-bit connection identity in context keys and rows; 0 = none */
static __always_inline __u32 mislo_conn32(__u64 key)
{
	return key ? ((__u32)(key ^ (key >> 32)) | 1u) : 0u;
}

/* the trace id the kernel assigns for its `fresh`-th new trace hash (wraps in 1 .. 2^24 - 1) */
static __always_inline __u32 mislo_trace_slot(__u64 fresh)
{
	return (__u32)(fresh % (MISLO_KERNEL_TRACE_LIMIT - 1)) + 1;
}

/* value_milli = raw * 10^shift: the catalogue's decode scales are powers of ten
 * (signals/catalog.py decode_scale; records.py milli_shift_table is the same table). */
static __always_inline int mislo_milli_shift(__u16 type)
{
	switch (type) {
	case MISLO_DNS_LATENCY: case MISLO_RUNQUEUE_DELAY: case MISLO_CONNECT_LATENCY:
	case MISLO_TLS_HANDSHAKE: case MISLO_MEM_RECLAIM: case MISLO_DISK_IO_LATENCY:
	case MISLO_SYSCALL_LATENCY: case MISLO_CFS_THROTTLE: case MISLO_GPU_QUEUE_DELAY:
	case MISLO_RCCL_COLLECTIVE:
		return -3; /* ns -> ms */
	case MISLO_CPU_STEAL: case MISLO_HBM_PRESSURE: case MISLO_XGMI_LATENCY:
		return 0;  /* milli-percent -> percent, ns -> us */
	default:
		return 3;  /* counts */
	}
}

/* records.py milli_int: half-to-even rounding, saturated to u32; integer-only (BPF has no
 * floating point). */
static __always_inline __u32 mislo_milli(__u16 type, __u64 v)
{
	int d = mislo_milli_shift(type);
	if (d == 3)
		return v > 4294967ull ? 0xFFFFFFFFu : (__u32)(v * 1000);
	if (d == 0)
		return v > 0xFFFFFFFFull ? 0xFFFFFFFFu : (__u32)v;
	__u64 q = v / 1000, r = v % 1000;
	q += (2 * r > 1000) || (2 * r == 1000 && (q & 1));
	return q > 0xFFFFFFFFull ? 0xFFFFFFFFu : (__u32)q;
}

#endif /* MISLO_RECORD_H */
