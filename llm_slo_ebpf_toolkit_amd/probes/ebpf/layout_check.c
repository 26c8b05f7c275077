/* Host-side check that struct mislo_event / mislo_event16 / mislo_def16 match
 * collector/records.py EVENT / EVENT16 / DEF_*, and that mislo_milli, mislo_conn32 and
 * mislo_trace_slot agree with records.py milli_int / conn32 / the trace-id wrap on boundary
 * values (the Python side compares the printed rows). */
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
	if (sizeof(struct mislo_event16) != 16 || offsetof(struct mislo_event16, ts_off) != 0 ||
	    offsetof(struct mislo_event16, ctx_type) != 4 || offsetof(struct mislo_event16, value_milli) != 8 ||
	    offsetof(struct mislo_event16, trace_tag) != 12) {
		printf("bad mislo_event16 layout\n");
		return 1;
	}
	if (sizeof(struct mislo_def16) != 16 || offsetof(struct mislo_def16, tag_id) != 4) {
		printf("bad mislo_def16 layout\n");
		return 1;
	}
	if (sizeof(struct mislo_batch) != 16 * MISLO_BATCH_SLOTS || MISLO_BATCH_SLOTS != 8) {
		printf("bad mislo_batch layout\n");
		return 1;
	}
	printf("mislo_event layout ok (64 bytes), mislo_event16 ok (16 bytes), mislo_def16 ok (16 bytes)\n");
	printf("const %u %u %u %u %u\n", MISLO_DEF_FIRST, MISLO_DEF_TRACE, MISLO_DEF_CTX, MISLO_KERNEL_CTX_LIMIT,
	       MISLO_KERNEL_TRACE_LIMIT);
	/* fixed-point rule: print "type value milli" lines for the Python side to compare */
	static const unsigned long long vals[] = {0, 499, 500, 501, 1500, 2500, 2501, 4294967, 4294968,
						   4294967295ull, 4294967296ull, 4294967295500ull, 4294967296500ull};
	static const unsigned short types[] = {MISLO_DNS_LATENCY, MISLO_TCP_RETRANSMIT, MISLO_CPU_STEAL, 99};
	for (unsigned t = 0; t < sizeof(types) / sizeof(types[0]); ++t)
		for (unsigned i = 0; i < sizeof(vals) / sizeof(vals[0]); ++i)
			printf("milli %u %llu %u\n", types[t], vals[i], mislo_milli(types[t], vals[i]));
	static const unsigned long long keys[] = {0, 1, 0xFFFFFFFFull, 0x100000000ull, 0x123456789ABCDEF0ull,
						   0xFFFFFFFFFFFFFFFFull, 0x8000000000000001ull};
	for (unsigned i = 0; i < sizeof(keys) / sizeof(keys[0]); ++i)
		printf("conn32 %llu %u\n", keys[i], mislo_conn32(keys[i]));
	static const unsigned long long fresh[] = {0, 1, (1ull << 29) - 3, (1ull << 29) - 2, (1ull << 29) - 1,
						    1ull << 29, 1ull << 33};
	for (unsigned i = 0; i < sizeof(fresh) / sizeof(fresh[0]); ++i)
		printf("trace %llu %u\n", fresh[i], mislo_trace_slot(fresh[i]));
	return 0;
}
