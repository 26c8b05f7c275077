/* Host build of the probes' shared BPF plumbing: compiles mislo_probe.h as written (the
 * interning with definitions ahead of map inserts, the epoch-offset packing, the emit floors,
 * the per-CPU staging batches) against in-process maps, and runs mislo_emit's logic over a file
 * of 64-byte mislo_event records. The batches it "puts on the ring" go to the output file, 128
 * bytes each (8 slots), so the tests compare the C the kernel runs with the runtime's ProbeSim
 * (runtime/csrc/probesim.cpp) and the numpy ProbeModel (collector/records.py) batch for batch.
 * A record's CPU is its tid % HOST_CPUS (ProbeSim's model of the task's CPU).
 *
 *   probe_host IN OUT [--epoch-at IDX:VALUE]... [--trace-next N] [--ctx-next N]
 *                     [--floor TYPE:VALUE]... [--ring-cap BATCHES] [--shard POD:SHARD]...
 *
 * --epoch-at is the agent's window cut before input record IDX: mislo_cfg[124] = VALUE, then
 * mislo_flush.bpf.c on every CPU in turn; the end of the input is a last cut (flush only);
 * --ring-cap makes bpf_ringbuf_output fail once that many batches are out (a full ring);
 * --shard routes a pod's records to split ring SHARD (mislo_shards), written to OUT.SHARD. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mislo_probe.h"

/* ---- maps ----------------------------------------------------------------------------- */
struct hmap {
	unsigned key_size, cap;
	unsigned char *keys;
	__u32 *vals;
	unsigned char *used;
};

#define HOST_CPUS 16
static struct hmap traces_m, ctxs_m, pods_m, shards_m;
static __u64 cfg_m[MISLO_CFG_SLOTS];
static struct mislo_event scratch_m;
static struct mislo_stage stages_m[HOST_CPUS][MISLO_SHARDS];
static unsigned cur_cpu;
static FILE *ring_out, *shard_out[MISLO_SHARDS];
static const char *out_path;
static unsigned long long ring_n, ring_cap = ~0ull;

static void hmap_init(struct hmap *m, unsigned key_size, unsigned cap)
{
	m->key_size = key_size;
	m->cap = cap;
	m->keys = calloc((size_t)cap, key_size);
	m->vals = calloc((size_t)cap, sizeof(__u32));
	m->used = calloc((size_t)cap, 1);
	if (!m->keys || !m->vals || !m->used) {
		fprintf(stderr, "out of memory\n");
		exit(2);
	}
}

static unsigned hmap_slot(const struct hmap *m, const void *key, int *found)
{
	__u64 h = 1469598103934665603ull;
	for (unsigned i = 0; i < m->key_size; ++i)
		h = (h ^ ((const unsigned char *)key)[i]) * 1099511628211ull;
	for (unsigned s = (unsigned)h & (m->cap - 1);; s = (s + 1) & (m->cap - 1)) {
		if (!m->used[s]) {
			*found = 0;
			return s;
		}
		if (!memcmp(m->keys + (size_t)s * m->key_size, key, m->key_size)) {
			*found = 1;
			return s;
		}
	}
}

static struct hmap *hmap_of(void *map)
{
	if (map == (void *)&mislo_traces)
		return &traces_m;
	if (map == (void *)&mislo_ctxs)
		return &ctxs_m;
	if (map == (void *)&mislo_pods)
		return &pods_m;
	if (map == (void *)&mislo_shards)
		return &shards_m;
	return 0;
}

void *bpf_map_lookup_elem(void *map, const void *key)
{
	__u32 idx = *(const __u32 *)key;
	if (map == (void *)&mislo_cfg)
		return idx < MISLO_CFG_SLOTS ? &cfg_m[idx] : 0;
	if (map == (void *)&mislo_scratch)
		return idx == 0 ? &scratch_m : 0;
	if (map == (void *)&mislo_stages)
		return idx < MISLO_SHARDS ? &stages_m[cur_cpu][idx] : 0;
	struct hmap *m = hmap_of(map);
	if (!m)
		return 0;
	int found;
	unsigned s = hmap_slot(m, key, &found);
	return found ? &m->vals[s] : 0;
}

long bpf_map_update_elem(void *map, const void *key, const void *value, __u64 flags)
{
	struct hmap *m = hmap_of(map);
	if (!m)
		return -22;
	int found;
	unsigned s = hmap_slot(m, key, &found);
	if (found && flags == BPF_NOEXIST)
		return -17;
	if (!found && flags == BPF_EXIST)
		return -2;
	memcpy(m->keys + (size_t)s * m->key_size, key, m->key_size);
	m->vals[s] = *(const __u32 *)value;
	m->used[s] = 1;
	return 0;
}

static int shard_of_ring(void *ringbuf)
{
	if (ringbuf == (void *)&mislo_events)
		return 0;
#if MISLO_SHARDS > 1
	if (ringbuf == (void *)&mislo_events1)
		return 1;
#endif
#if MISLO_SHARDS > 2
	if (ringbuf == (void *)&mislo_events2)
		return 2;
#endif
#if MISLO_SHARDS > 3
	if (ringbuf == (void *)&mislo_events3)
		return 3;
#endif
#if MISLO_SHARDS > 4
	if (ringbuf == (void *)&mislo_events4)
		return 4;
	if (ringbuf == (void *)&mislo_events5)
		return 5;
	if (ringbuf == (void *)&mislo_events6)
		return 6;
	if (ringbuf == (void *)&mislo_events7)
		return 7;
#endif
	return -1;
}

long bpf_ringbuf_output(void *ringbuf, void *data, __u64 size, __u64 flags)
{
	(void)flags;
	int s = shard_of_ring(ringbuf);
	if (s < 0 || size != MISLO_BATCH_BYTES)
		return -22;
	if (ring_n >= ring_cap)
		return -11; /* -EAGAIN: ring full */
	FILE *f = ring_out;
	if (s > 0) {
		if (!shard_out[s]) {
			char p[4096];
			snprintf(p, sizeof(p), "%s.%d", out_path, s);
			shard_out[s] = fopen(p, "wb");
			if (!shard_out[s])
				return -5;
		}
		f = shard_out[s];
	}
	if (fwrite(data, MISLO_BATCH_BYTES, 1, f) != 1)
		return -5;
	++ring_n;
	return 0;
}

__u64 bpf_ktime_get_ns(void) { return 0; }
__u64 bpf_get_current_cgroup_id(void) { return 0; }
__u64 bpf_get_current_pid_tgid(void) { return 0; }

/* ---- driver --------------------------------------------------------------------------- */
struct epoch_at {
	unsigned long long idx, value;
};

int main(int argc, char **argv)
{
	if (argc < 3) {
		fprintf(stderr, "usage: probe_host IN OUT [--epoch-at IDX:VALUE]... [--trace-next N] "
				"[--ctx-next N] [--floor TYPE:VALUE]... [--ring-cap N]\n");
		return 2;
	}
	static struct epoch_at ep[4096];
	unsigned n_ep = 0;
	for (int i = 3; i + 1 < argc; i += 2) {
		unsigned long long a, b;
		if (!strcmp(argv[i], "--epoch-at") && sscanf(argv[i + 1], "%llu:%llu", &a, &b) == 2 && n_ep < 4096)
			ep[n_ep].idx = a, ep[n_ep++].value = b;
		else if (!strcmp(argv[i], "--trace-next"))
			cfg_m[MISLO_CFG_TRACE_NEXT] = strtoull(argv[i + 1], 0, 0);
		else if (!strcmp(argv[i], "--ctx-next"))
			cfg_m[MISLO_CFG_CTX_NEXT] = strtoull(argv[i + 1], 0, 0);
		else if (!strcmp(argv[i], "--floor") && sscanf(argv[i + 1], "%llu:%llu", &a, &b) == 2 && a < 120)
			cfg_m[MISLO_CFG_FLOOR(a)] = b;
		else if (!strcmp(argv[i], "--ring-cap"))
			ring_cap = strtoull(argv[i + 1], 0, 0);
		else if (!strcmp(argv[i], "--shard") && sscanf(argv[i + 1], "%llu:%llu", &a, &b) == 2) {
			if (!shards_m.cap)
				hmap_init(&shards_m, 4, 1u << 16);
			__u32 pod = (__u32)a, sh = (__u32)b;
			bpf_map_update_elem(&mislo_shards, &pod, &sh, BPF_ANY);
		}
		else {
			fprintf(stderr, "bad option %s\n", argv[i]);
			return 2;
		}
	}
	if (!shards_m.cap)
		hmap_init(&shards_m, 4, 1u << 16);
	hmap_init(&traces_m, 8, 1u << 22);
	hmap_init(&ctxs_m, sizeof(struct mislo_ctx_key), 1u << 22);
	hmap_init(&pods_m, 8, 1u << 16);
	FILE *in = fopen(argv[1], "rb");
	out_path = argv[2];
	ring_out = fopen(argv[2], "wb");
	if (!in || !ring_out) {
		perror("open");
		return 2;
	}
	for (unsigned c = 0; c < HOST_CPUS; ++c)
		for (unsigned sh = 0; sh < MISLO_SHARDS; ++sh)
			mislo_pad_batch(&stages_m[c][sh].b);
	struct mislo_event ev;
	unsigned long long n = 0;
	unsigned e = 0;
	while (fread(&ev, sizeof(ev), 1, in) == 1) {
		while (e < n_ep && ep[e].idx <= n) { /* the agent's cut: epoch, then every CPU's flush */
			cfg_m[MISLO_CFG_EPOCH] = ep[e++].value;
			for (cur_cpu = 0; cur_cpu < HOST_CPUS; ++cur_cpu)
				mislo_flush_cpu();
		}
		/* mislo_emit with the record's own task / pod on its CPU: the floor, then the working record */
		cur_cpu = ev.tid % HOST_CPUS;
		if (!mislo_below_floor(ev.signal_type, ev.value)) {
			scratch_m = ev;
			mislo_submit(&scratch_m);
		}
		++n;
	}
	for (cur_cpu = 0; cur_cpu < HOST_CPUS; ++cur_cpu)
		mislo_flush_cpu();
	fclose(in);
	fclose(ring_out);
	for (int s = 1; s < MISLO_SHARDS; ++s)
		if (shard_out[s])
			fclose(shard_out[s]);
	printf("events %llu batches %llu trace_next %llu ctx_next %llu\n", n, ring_n,
	       (unsigned long long)cfg_m[MISLO_CFG_TRACE_NEXT], (unsigned long long)cfg_m[MISLO_CFG_CTX_NEXT]);
	return 0;
}
