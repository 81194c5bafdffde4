/* TEST ONLY (tests/test_real_headers.py).  Stand-in for the header libevent's
 * configure generates (the reference vendors libevent's sources, not it). */
#ifndef _EVENT2_EVENT_CONFIG_H_
#define _EVENT2_EVENT_CONFIG_H_
#define _EVENT_HAVE_SYS_TYPES_H 1
#define _EVENT_HAVE_SYS_TIME_H 1
#define _EVENT_HAVE_STDINT_H 1
#define _EVENT_HAVE_INTTYPES_H 1
#define _EVENT_HAVE_UNISTD_H 1
#define _EVENT_HAVE_STDDEF_H 1
#define _EVENT_HAVE_SYS_SOCKET_H 1
#define _EVENT_HAVE_NETINET_IN_H 1
#define _EVENT_HAVE_UINT64_T 1
#define _EVENT_HAVE_UINT32_T 1
#define _EVENT_HAVE_UINT16_T 1
#define _EVENT_HAVE_UINT8_T 1
#define _EVENT_HAVE_UINTPTR_T 1
#define _EVENT_SIZEOF_LONG 8
#define _EVENT_SIZEOF_LONG_LONG 8
#define _EVENT_SIZEOF_INT 4
#define _EVENT_SIZEOF_SHORT 2
#define _EVENT_SIZEOF_SIZE_T 8
#define _EVENT_SIZEOF_VOID_P 8
#define _EVENT_SIZEOF_OFF_T 8
#define _EVENT_HAVE_FD_MASK 1
#define _EVENT_HAVE_TIMERADD 1
#define _EVENT_HAVE_TIMERCLEAR 1
#define _EVENT_HAVE_TIMERCMP 1
#define _EVENT_HAVE_TIMERISSET 1
#define _EVENT_ssize_t ssize_t
#define _EVENT_DISABLE_THREAD_SUPPORT 0
#define _EVENT_HAVE_PTHREADS 1
#endif
