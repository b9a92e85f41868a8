/*
 * niperrorhandler.h -- drop-in for the reference's src/niperrorhandler.h
 * (nip_amd compat layer, libnip.so).  The NIP_ERROR_* codes come from
 * include/nip_amd.h, which takes the reference's values.
 */
#ifndef NIP_AMD_COMPAT_ERRORHANDLER_H
#define NIP_AMD_COMPAT_ERRORHANDLER_H

#include "nip_amd.h" /* NIP_NO_ERROR, NIP_ERROR_* */

#ifdef __cplusplus
extern "C" {
#endif

/* src/niperrorhandler.c: prints "In <file> (<line>): <message>" on stderr
 * when verbose, remembers the code, counts the call and returns error. */
int nip_report_error(char* srcFile, int line, int error, int verbose);
void nip_reset_error_handler(void);
int nip_check_error_type(void);
int nip_check_error_counter(void);

#ifdef __cplusplus
}
#endif
#endif
