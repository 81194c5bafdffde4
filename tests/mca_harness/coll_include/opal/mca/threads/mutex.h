/* TEST HARNESS ONLY: opal_mutex_t over pthreads (opal/mca/threads/mutex.h:118). */
#ifndef HARNESS_OPAL_MUTEX_H
#define HARNESS_OPAL_MUTEX_H
#include <pthread.h>
typedef struct opal_mutex_t { pthread_mutex_t m; } opal_mutex_t;
#define OPAL_MUTEX_STATIC_INIT {PTHREAD_MUTEX_INITIALIZER}
#define OPAL_THREAD_LOCK(mx) pthread_mutex_lock(&(mx)->m)
#define OPAL_THREAD_UNLOCK(mx) pthread_mutex_unlock(&(mx)->m)
#endif
