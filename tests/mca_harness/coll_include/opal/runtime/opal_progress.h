/* TEST HARNESS ONLY: progress-callback registration
 * (opal/runtime/opal_progress.h:139-167). */
#ifndef HARNESS_OPAL_PROGRESS_H
#define HARNESS_OPAL_PROGRESS_H
typedef int (*opal_progress_callback_t)(void);
int opal_progress_register(opal_progress_callback_t cb);
int opal_progress_unregister(opal_progress_callback_t cb);
void opal_progress(void);
#endif
