/* 64-byte event record shared by every probe, the rocprofiler tool, the native ring and
 * the GPU decode kernel (collector/records.py EVENT, ops/csrc/mislo_common.h Event).
 * Only fixed-width types, so it compiles for the BPF target and for the host layout test. */
#ifndef MISLO_RECORD_H
#define MISLO_RECORD_H

#include <linux/types.h>

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

#endif /* MISLO_RECORD_H */
