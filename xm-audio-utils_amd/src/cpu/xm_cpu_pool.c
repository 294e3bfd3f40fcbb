/*
 * xm_cpu_pool.c — the CPU backend's worker threads (SURVEY.md §8(d) "OpenMP
 * over clips", done with plain pthreads so the library links no OpenMP
 * runtime).  One process-wide pool, created on first use: XM_CPU_THREADS
 * threads if set, else one per CPU of the process's affinity mask, the caller
 * counting as one.  Items (a mix and a range of its outputs, a clip, ...) are
 * handed out one at a time from an atomic counter, so uneven items balance.
 * One parallel region runs at a time; a region started while another runs
 * (another handle on another thread, or a nested call) runs on its caller.
 * Fork-safe: a child of fork() has none of the parent's workers, so the
 * child's first parallel region starts its own workers (Python
 * multiprocessing's fork start method after a CPU-backend call in the
 * parent).  pthread_atfork handlers, registered when the library loads, take
 * the region and worker locks around fork(): a fork() waits for a region (or
 * the pool's initialisation, which runs under the region lock) that another
 * thread is inside, and the child starts with both locks fresh.  Calling
 * fork() from inside a parallel region's item function is unsupported (it
 * would wait for its own region).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdlib.h>

#include "xm_cpu.h"

#define XMC_MAX_THREADS 512

static struct {
    _Atomic int ready;            /* 1: sized and workers started (cleared in a forked child) */
    int n;                        /* threads including the caller */
    int want;                     /* threads asked for (XM_CPU_THREADS or the affinity mask); 0: not sized yet */
    pthread_mutex_t mu, region;
    pthread_cond_t go, done;
    unsigned long gen;
    int busy;                     /* workers still inside the current region */
    XmcItemFn fn;
    void *ctx;
    int64_t n_items;
    _Atomic int64_t next;
} P = {0, 0, 0, PTHREAD_MUTEX_INITIALIZER, PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER,
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

/* start the workers (P.region held, no worker running) */
static void spawn_workers(void)
{
    P.n = 1;
    for (int i = 1; i < P.want; ++i) {
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

/* fork(): no region and no initialisation in flight while the address space
 * is copied; the parent carries on, the child has only the forking thread
 * (the parent's workers are gone) and fresh locks */
static void atfork_prepare(void)
{
    pthread_mutex_lock(&P.region);
    pthread_mutex_lock(&P.mu);
}

static void atfork_parent(void)
{
    pthread_mutex_unlock(&P.mu);
    pthread_mutex_unlock(&P.region);
}

static void atfork_child(void)
{
    pthread_mutex_init(&P.mu, NULL);
    pthread_mutex_init(&P.region, NULL);
    pthread_cond_init(&P.go, NULL);
    pthread_cond_init(&P.done, NULL);
    P.gen = 0;
    P.busy = 0;
    P.n = 1;
    atomic_store(&P.ready, 0);   /* the first region starts the child's own workers */
}

__attribute__((constructor)) static void register_atfork(void)
{
    pthread_atfork(atfork_prepare, atfork_parent, atfork_child);
}

/* size the pool on first use and start its workers (again in a forked child) */
static void ensure_pool(void)
{
    if (atomic_load(&P.ready)) return;
    pthread_mutex_lock(&P.region);
    if (!atomic_load(&P.ready)) {
        if (!P.want) {
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
            P.want = n;
        }
        spawn_workers();
        atomic_store(&P.ready, 1);
    }
    pthread_mutex_unlock(&P.region);
}

int xmc_threads(void)
{
    ensure_pool();
    return P.n;
}

int xmc_parallel(int64_t n, XmcItemFn fn, void *ctx)
{
    if (n <= 0) return 0;
    ensure_pool();
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
