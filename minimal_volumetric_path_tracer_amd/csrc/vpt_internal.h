/* vpt_internal.h -- shared host-side helpers of libvpt (not part of the ABI). */
#ifndef VPT_INTERNAL_H
#define VPT_INTERNAL_H

#include "../../include/vpt.h"

/* records a thread-local message for vpt_last_error() and returns `code` */
int vpt_fail(int code, const char* fmt, ...);
void vpt_clear_error(void);

#endif
