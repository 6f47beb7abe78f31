/* mamg_test.h -- test and verification hooks of libmamg.so.
 *
 * Not part of the preconditioner API (include/mamg.h): no reference
 * counterpart, no stability promise.  The tests and the A/B scripts use them;
 * a caller of the metric_mono path never needs them. */
#ifndef MAMG_TEST_H
#define MAMG_TEST_H
#include "mamg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Set (value != NULL)
 * or reset (NULL) one of the library's internal layout switches for the
 * process (names in mamg_option_names(); DESIGN.md section 4 gives the
 * measured defaults).  The product library reads no environment variables;
 * MAMG_ERR_ARG for an unknown name. */
int mamg_set_option(const char* name, const char* value);
const char* mamg_option_names(void);   /* comma-separated */

/* Verification of a row-sharded Galerkin product (the start of a
 * partition-local setup): on nranks
 * virtual ranks (fine nodes and coarse nodes split into even ranges), rank p
 * forms its (A P) rows from its A rows and the P rows of the fine dofs they
 * reach (its own and a halo), then its coarse rows of R (A P), R = P^T, from
 * its R rows and the (A P) rows of the fine dofs those reach, each taken from
 * the owner rank's sharded result; the GPU setup's own SpGEMM throughout.
 * A, P, Ac: one level's field-major 2-function operator, prolongator and the
 * hierarchy's next-level operator (host CSR).  res6: (A P) rows differing
 * from the unsharded product, A_c rows differing from Ac (bitwise), halo P
 * rows read, halo (A P) rows read, (A P) rows and A_c rows compared. */
int mamg_sharded_galerkin_check(const mamg_csr* A, const mamg_csr* P, const mamg_csr* Ac, int nranks, int device,
                                int64_t* res6);

#ifdef __cplusplus
}
#endif
#endif /* MAMG_TEST_H */
