/*
 * xm_pool.c — the host worker pool of the multi-device handles (SURVEY.md
 * §8(b): "a handle spawns one host worker thread per GPU, joined before
 * process_batch returns").  Worker d runs task(ctx, d, arg) once per dispatch
 * and the dispatching thread waits for all of them; with n == 1 the task runs
 * on the caller's thread.  Used by the mixer (src/xm_mixer_multi.c) and the
 * effects chain (src/xm_effects.c).
 */
#include <pthread.h>
#include <stdlib.h>

#include "xm_internal.h"

typedef struct XmPoolWorker {
    XmPool *p;
    int d;
} XmPoolWorker;

struct XmPool {
    int n;
    void *ctx;
    pthread_t th[XM_MAX_DEVICES];
    XmPoolWorker wk[XM_MAX_DEVICES];
    int n_threads;
    pthread_mutex_t lock;
    pthread_cond_t go, done;
    unsigned long gen;
    int pending, quit;
    XmPoolTask task;
    void *arg;
    int rc[XM_MAX_DEVICES];
};

static void *worker_main(void *q)
{
    XmPoolWorker *w = q;
    XmPool *p = w->p;
    unsigned long seen = 0;
    pthread_mutex_lock(&p->lock);
    for (;;) {
        while (!p->quit && p->gen == seen) pthread_cond_wait(&p->go, &p->lock);
        if (p->quit) break;
        seen = p->gen;
        XmPoolTask t = p->task;
        void *a = p->arg;
        pthread_mutex_unlock(&p->lock);
        int rc = t(p->ctx, w->d, a);
        pthread_mutex_lock(&p->lock);
        p->rc[w->d] = rc;
        if (--p->pending == 0) pthread_cond_signal(&p->done);
    }
    pthread_mutex_unlock(&p->lock);
    return NULL;
}

XmPool *xm_pool_create(int n, void *ctx, int *status)
{
    int rc = XM_OK;
    XmPool *p = NULL;
    if (n < 1 || n > XM_MAX_DEVICES) {
        rc = XM_EINVAL;
        goto out;
    }
    p = calloc(1, sizeof *p);
    if (!p) {
        rc = XM_ENOMEM;
        goto out;
    }
    p->n = n;
    p->ctx = ctx;
    pthread_mutex_init(&p->lock, NULL);
    pthread_cond_init(&p->go, NULL);
    pthread_cond_init(&p->done, NULL);
    for (int d = 0; d < n && n > 1; ++d) {
        p->wk[d].p = p;
        p->wk[d].d = d;
        if (pthread_create(&p->th[d], NULL, worker_main, &p->wk[d])) {
            rc = XM_ENOMEM;
            break;
        }
        p->n_threads++;
    }
    if (rc) xm_pool_free(&p);
out:
    if (status) *status = rc;
    return p;
}

void xm_pool_free(XmPool **pp)
{
    if (!pp || !*pp) return;
    XmPool *p = *pp;
    pthread_mutex_lock(&p->lock);
    p->quit = 1;
    pthread_cond_broadcast(&p->go);
    pthread_mutex_unlock(&p->lock);
    for (int d = 0; d < p->n_threads; ++d) pthread_join(p->th[d], NULL);
    pthread_cond_destroy(&p->go);
    pthread_cond_destroy(&p->done);
    pthread_mutex_destroy(&p->lock);
    free(p);
    *pp = NULL;
}

int xm_pool_run(XmPool *p, XmPoolTask t, void *arg)
{
    if (p->n_threads == 0) {
        for (int d = 0; d < p->n; ++d) p->rc[d] = t(p->ctx, d, arg);
    } else {
        pthread_mutex_lock(&p->lock);
        p->task = t;
        p->arg = arg;
        p->pending = p->n;
        p->gen++;
        pthread_cond_broadcast(&p->go);
        while (p->pending) pthread_cond_wait(&p->done, &p->lock);
        pthread_mutex_unlock(&p->lock);
    }
    for (int d = 0; d < p->n; ++d)
        if (p->rc[d]) return p->rc[d];
    return XM_OK;
}

void xm_block(size_t batch, int n, int d, size_t *first, size_t *cnt)
{
    const size_t q = batch / (size_t)n, r = batch % (size_t)n;
    *first = (size_t)d * q + ((size_t)d < r ? (size_t)d : r);
    *cnt = q + ((size_t)d < r ? 1 : 0);
}
