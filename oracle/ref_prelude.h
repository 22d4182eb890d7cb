/*
 * oracle/ref_prelude.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Prepended (by oracle/Makefile, through a pipe into gcc) to the hot-path lines
 * of the reference's own /root/reference/src/pg.c:104-179 (helpers,
 * reduce_inplace, pg_sendrecv_mock) and :264-339 (pg_reduce_scatter,
 * pg_all_gather, pg_all_reduce).  Those lines use only libc and the reference's
 * own include/pg.h, so they compile as-is: no stand-in header or library is
 * involved (connect_process_group / pg_close, which need libibverbs, are not
 * part of the extracted ranges).  No reference text is written into this repo;
 * only the compiled oracle/_ref/libpgref.so is produced (git-ignored).
 *
 * The exported reference symbols are renamed (-D) so they cannot collide with
 * the product library's pg_* if both are loaded into one process.
 */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include "pg.h"
