/*
 * xm_cpu_pool.c — the CPU backend's worker threads (SURVEY.md §8(d) "OpenMP
 * over clips", done with plain pthreads so the library links no OpenMP
 * runtime).  One process-wide pool, created on first use: XM_CPU_THREADS
 * threads if set, else one per CPU of the process's affinity mask, the caller
 * counting as one.  Items (a mix and a range of its outputs, a clip, ...) are
 * handed out one at a time from an atomic counter, so uneven items balance.
 * One parallel region runs at a time; a region started while another runs
 * (another handle on another thread, or a nested call) runs on its caller.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdlib.h>

#include "xm_cpu.h"

#define XMC_MAX_THREADS 512

static struct {
    pthread_once_t once;
    int n;                        /* threads including the caller */
    pthread_mutex_t mu, region;
    pthread_cond_t go, done;
    unsigned long gen;
    int busy;                     /* workers still inside the current region */
    XmcItemFn fn;
    void *ctx;
    int64_t n_items;
    _Atomic int64_t next;
} P = {PTHREAD_ONCE_INIT, 0, PTHREAD_MUTEX_INITIALIZER, PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER,
       PTHREAD_COND_INITIALIZER, 0, 0, NULL, NULL, 0, 0};

static void drain(XmcItemFn fn, void *ctx, int64_t n)
{
    for (;;) {
        const int64_t i = atomic_fetch_add_explicit(&P.next, 1, memory_order_relaxed);
        if (i >= n) return;
        fn(ctx, i);
    }
}

static void *worker(void *arg)
{
    (void)arg;
    unsigned long seen = 0;
    pthread_mutex_lock(&P.mu);
    for (;;) {
        while (P.gen == seen) pthread_cond_wait(&P.go, &P.mu);
        seen = P.gen;
        XmcItemFn fn = P.fn;
        void *ctx = P.ctx;
        const int64_t n = P.n_items;
        pthread_mutex_unlock(&P.mu);
        drain(fn, ctx, n);
        pthread_mutex_lock(&P.mu);
        if (--P.busy == 0) pthread_cond_signal(&P.done);
    }
    return NULL;
}

static void init_pool(void)
{
    int n = 0;
    const char *e = getenv("XM_CPU_THREADS");
    if (e && atoi(e) > 0) {
        n = atoi(e);
    } else {
        cpu_set_t set;
        if (sched_getaffinity(0, sizeof set, &set) == 0) n = CPU_COUNT(&set);
    }
    if (n < 1) n = 1;
    if (n > XMC_MAX_THREADS) n = XMC_MAX_THREADS;
    P.n = 1;
    for (int i = 1; i < n; ++i) {
        pthread_t t;
        pthread_attr_t at;
        pthread_attr_init(&at);
        pthread_attr_setdetachstate(&at, PTHREAD_CREATE_DETACHED);
        const int rc = pthread_create(&t, &at, worker, NULL);
        pthread_attr_destroy(&at);
        if (rc) break;   /* fewer threads than asked: still correct */
        P.n++;
    }
}

int xmc_threads(void)
{
    pthread_once(&P.once, init_pool);
    return P.n;
}

int xmc_parallel(int64_t n, XmcItemFn fn, void *ctx)
{
    if (n <= 0) return 0;
    pthread_once(&P.once, init_pool);
    if (P.n == 1 || n == 1 || pthread_mutex_trylock(&P.region) != 0) {
        for (int64_t i = 0; i < n; ++i) fn(ctx, i);   /* serial: one item, one thread, or the pool is busy */
        return 0;
    }
    pthread_mutex_lock(&P.mu);
    P.fn = fn;
    P.ctx = ctx;
    P.n_items = n;
    atomic_store_explicit(&P.next, 0, memory_order_relaxed);
    P.busy = P.n - 1;
    P.gen++;
    pthread_cond_broadcast(&P.go);
    pthread_mutex_unlock(&P.mu);
    drain(fn, ctx, n);
    pthread_mutex_lock(&P.mu);
    while (P.busy) pthread_cond_wait(&P.done, &P.mu);
    pthread_mutex_unlock(&P.mu);
    pthread_mutex_unlock(&P.region);
    return 0;
}
