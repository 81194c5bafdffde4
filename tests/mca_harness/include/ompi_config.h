/* TEST HARNESS ONLY: minimal stand-in for a configured Open MPI tree's
 * ompi_config.h, enough to compile ompi_amd/mca/op/rocm against.  The real
 * build uses the configured tree. */
#ifndef HARNESS_OMPI_CONFIG_H
#define HARNESS_OMPI_CONFIG_H
#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#define BEGIN_C_DECLS
#define END_C_DECLS
#define OMPI_DECLSPEC
#define OMPI_MODULE_DECLSPEC
#define OMPI_MAJOR_VERSION 5
#define OMPI_MINOR_VERSION 0
#define OMPI_RELEASE_VERSION 0
#endif
