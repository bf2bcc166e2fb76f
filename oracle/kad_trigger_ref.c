/* TEST INFRASTRUCTURE ONLY — CPU restatement of the FNV-1 half of
 * Scheduler.computeSchedulingTriggerHash (pkg/controllers/scheduler/
 * schedulingtriggers.go:141-145): hash/fnv.New32 (FNV-1, 32-bit; SURVEY.md
 * Appendix A.5) written with the object's trigger JSON. As in the reference,
 * every object hashes its own bytes end to end: object part, then the shared
 * cluster part — no state sharing between objects. Used by tests/ as the
 * checker of kad_trigger_* and by bench.py's cpu_baseline leg.             */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>

static uint32_t fnv1(uint32_t h, const uint8_t* p, int64_t n) {
  for (int64_t i = 0; i < n; i++) h = (h * 16777619u) ^ p[i];
  return h;
}

typedef struct {
  int begin, end, stride;
  const int64_t* off;
  const uint8_t *pre, *suf;
  int64_t suf_len;
  uint32_t* out;
} tjob_t;

static void* tworker(void* arg) {
  tjob_t* j = arg;
  for (int i = j->begin; i < j->end; i += j->stride) {
    uint32_t h = fnv1(2166136261u, j->pre + j->off[i], j->off[i + 1] - j->off[i]);
    j->out[i] = fnv1(h, j->suf, j->suf_len);
  }
  return NULL;
}

int kad_ref_trigger_hashes(int n, const int64_t* off, const uint8_t* prefix, const uint8_t* suffix, int64_t suffix_len,
                           uint32_t* out, int n_threads) {
  if (n < 0) return -1;
  if (n_threads < 1) n_threads = 1;
  pthread_t* th = malloc(sizeof(pthread_t) * n_threads);
  tjob_t* jobs = malloc(sizeof(tjob_t) * n_threads);
  int* started = calloc(n_threads, sizeof(int));
  for (int t = 0; t < n_threads; t++) jobs[t] = (tjob_t){t, n, n_threads, off, prefix, suffix, suffix_len, out};
  for (int t = 0; t < n_threads; t++) {
    if (n_threads > 1 && pthread_create(&th[t], NULL, tworker, &jobs[t]) == 0) started[t] = 1;
    else tworker(&jobs[t]);
  }
  for (int t = 0; t < n_threads; t++) if (started[t]) pthread_join(th[t], NULL);
  free(started);
  free(th);
  free(jobs);
  return 0;
}
