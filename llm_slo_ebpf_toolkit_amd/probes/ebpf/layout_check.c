/* Host-side check that struct mislo_event / mislo_event32 / mislo_event24 / mislo_event20t match
 * collector/records.py EVENT / EVENT32 / EVENT24 / EVENT20T, and that mislo_milli agrees with records.py milli_int on boundary values. */
#include <stddef.h>
#include <stdio.h>

#include "mislo_record.h"

#define CHECK(field, off)                                                                   \
	do {                                                                                    \
		if (offsetof(struct mislo_event, field) != (off)) {                                  \
			printf("bad offset %s: %zu != %d\n", #field, offsetof(struct mislo_event, field), off); \
			return 1;                                                                       \
		}                                                                                   \
	} while (0)

int main(void)
{
	if (sizeof(struct mislo_event) != 64) {
		printf("bad size %zu\n", sizeof(struct mislo_event));
		return 1;
	}
	CHECK(ts_ns, 0); CHECK(value, 8); CHECK(trace_h, 16); CHECK(pid, 24); CHECK(tid, 28);
	CHECK(pod_id, 32); CHECK(dst_ip, 36); CHECK(signal_type, 40); CHECK(node_id, 42);
	CHECK(svc_id, 44); CHECK(flags, 46); CHECK(src_port, 48); CHECK(dst_port, 50);
	CHECK(err, 52); CHECK(conn_h, 56);
	if (sizeof(struct mislo_event32) != 32) {
		printf("bad size %zu\n", sizeof(struct mislo_event32));
		return 1;
	}
#define CHECK32(field, off)                                                                  \
	do {                                                                                    \
		if (offsetof(struct mislo_event32, field) != (off)) {                                \
			printf("bad offset %s\n", #field);                                              \
			return 1;                                                                       \
		}                                                                                   \
	} while (0)
	CHECK32(ts_ns, 0); CHECK32(trace_h, 8); CHECK32(value_milli, 16); CHECK32(pid, 20);
	CHECK32(pod_id, 24); CHECK32(type_conn, 28);
	if (sizeof(struct mislo_event24) != 24 || offsetof(struct mislo_event24, ts_ns) != 0 ||
	    offsetof(struct mislo_event24, trace_h) != 8 || offsetof(struct mislo_event24, value_milli) != 16 ||
	    offsetof(struct mislo_event24, ctx_type) != 20) {
		printf("bad mislo_event24 layout\n");
		return 1;
	}
	if (sizeof(struct mislo_event20t) != 20 || offsetof(struct mislo_event20t, ts_ns) != 0 ||
	    offsetof(struct mislo_event20t, value_milli) != 8 || offsetof(struct mislo_event20t, ctx_type) != 12 ||
	    offsetof(struct mislo_event20t, trace_id) != 16 || _Alignof(struct mislo_event20t) != 4) {
		printf("bad mislo_event20t layout\n");
		return 1;
	}
	if (sizeof(struct mislo_event16) != 16 || offsetof(struct mislo_event16, ts_off) != 0 ||
	    offsetof(struct mislo_event16, ctx_type) != 4 || offsetof(struct mislo_event16, value_milli) != 8 ||
	    offsetof(struct mislo_event16, trace_tag) != 12) {
		printf("bad mislo_event16 layout\n");
		return 1;
	}
	printf("mislo_event layout ok (64 bytes), mislo_event32 ok (32 bytes), mislo_event24 ok (24 bytes), "
	       "mislo_event20t ok (20 bytes), mislo_event16 ok (16 bytes)\n");
	/* fixed-point rule: print "type value milli" lines for the Python side to compare */
	static const unsigned long long vals[] = {0, 499, 500, 501, 1500, 2500, 2501, 4294967, 4294968,
						   4294967295ull, 4294967296ull, 4294967295500ull, 4294967296500ull};
	static const unsigned short types[] = {MISLO_DNS_LATENCY, MISLO_TCP_RETRANSMIT, MISLO_CPU_STEAL, 99};
	for (unsigned t = 0; t < sizeof(types) / sizeof(types[0]); ++t)
		for (unsigned i = 0; i < sizeof(vals) / sizeof(vals[0]); ++i)
			printf("milli %u %llu %u\n", types[t], vals[i], mislo_milli(types[t], vals[i]));
	return 0;
}
