/* Event records shared by the probes, the rocprofiler tool, the native ring and the GPU
 * decode kernels. Only fixed-width types, so it compiles for the BPF target and for the host
 * layout test.
 *   struct mislo_event   (64 B, collector/records.py EVENT): the probes' working record and
 *                        the user-space producers' ring record;
 *   struct mislo_event20t (20 B, records.py EVENT20T): the ring record with
 *                        -DMISLO_RING_EVENT20T: mislo_event24 with the trace hash interned in the kernel
 *                        too (mislo_probe.h mislo_trace_id; the agent maps span trace ids
 *                        through the same map), 5/16 of the 64-byte record's PCIe bytes;
 *   struct mislo_event16 (16 B, records.py EVENT16): what the probes put on the BPF ring
 *                        (default): mislo_event20t with the timestamp as a 32-bit offset from the epoch the
 *                        agent last published (mislo_cfg[MISLO_CFG_EPOCH]) and that epoch's 2-bit
 *                        tag in the top of trace_id, so records emitted across a window cut
 *                        decode exactly (the window carries its last 4 epoch bases);
 *   struct mislo_event24 (24 B, records.py EVENT24): the ring record with -DMISLO_RING_EVENT24.
 *                        The kernel converts the value to fixed point
 *                        (mislo_milli) and interns the connection and the (pod, pid, conn)
 *                        context (mislo_probe.h mislo_conn_id / mislo_ctx_id), so the agent
 *                        DMAs ring bytes to the GPU without touching a record: 3/8 of the PCIe
 *                        bytes of the 64-byte record. The agent turns new context ids into
 *                        device context-table rows (adding svc / node from pod metadata);
 *   struct mislo_event32 (32 B, records.py EVENT32): the ring record with -DMISLO_RING_EVENT32
 *                        (connections interned, pod and pid inline; svc / node from the
 *                        agent's pod table). */
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

struct mislo_event32 {
	__s64 ts_ns;       /* CLOCK_REALTIME ns */
	__u64 trace_h;     /* trace-id hash (0 = none) */
	__u32 value_milli; /* value in 1/1000 of the signal's output unit (mislo_milli) */
	__u32 pid;         /* tgid */
	__u32 pod_id;      /* cgroup -> pod id, 0 = unknown */
	__u32 type_conn;   /* bits 0-7 signal type, bits 8-31 interned connection id (0 = none) */
};

struct mislo_event24 {
	__s64 ts_ns;       /* CLOCK_REALTIME ns */
	__u64 trace_h;     /* trace-id hash (0 = none) */
	__u32 value_milli; /* value in 1/1000 of the signal's output unit (mislo_milli) */
	__u32 ctx_type;    /* bits 0-7 signal type, bits 8-31 interned context id (0 = none) */
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

/* 4-byte aligned: ring records are packed back to back at 20-byte strides */
struct mislo_event20t {
	__s64 ts_ns;       /* CLOCK_REALTIME ns */
	__u32 value_milli; /* value in 1/1000 of the signal's output unit (mislo_milli) */
	__u32 ctx_type;    /* bits 0-7 signal type, bits 8-31 interned context id (0 = none) */
	__u32 trace_id;    /* interned trace id (mislo_trace_id), 0 = none */
} __attribute__((packed, aligned(4)));

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
