/* TEST HARNESS ONLY: the process name the coll glue reads. */
#ifndef HARNESS_OMPI_RTE_H
#define HARNESS_OMPI_RTE_H
typedef struct { unsigned jobid, vpid; } harness_proc_name_t;
extern harness_proc_name_t harness_proc_name;
#define OMPI_PROC_MY_NAME (&harness_proc_name)
#endif
