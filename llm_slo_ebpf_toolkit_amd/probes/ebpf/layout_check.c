/* Host-side check that struct mislo_event matches collector/records.py EVENT. */
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
	printf("mislo_event layout ok (64 bytes)\n");
	return 0;
}
