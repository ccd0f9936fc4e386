/* ElasticQuota admission: CPU restatement (TEST INFRASTRUCTURE ONLY — the checker for the GPU path,
 * never linked into libkoordeval).  See quota.c. */
#ifndef OR_QUOTA_H
#define OR_QUOTA_H
#include "koord_eval.h"

typedef struct or_quotas {
  int32_t n;
  ke_quota_args args;
  ke_quota q[KE_MAX_QUOTAS];
  int64_t limit[KE_MAX_QUOTAS][KE_NRES]; /* getQuotaInfoUsedLimit */
  uint8_t limit_has[KE_MAX_QUOTAS][KE_NRES];
} or_quotas;

int orq_load(or_quotas* Q, const ke_quota_args* args, const ke_quota* q, int32_t n);
/* PreFilter: -1 = Skip (no quota), 1 = admitted, 0 = Unschedulable */
int orq_admit(const or_quotas* Q, const ke_pod* pod);
void orq_reserve(or_quotas* Q, const ke_pod* pod);
/* Unreserve of an assigned pod (assigned) and/or its request leaving the tree (del, informer delete) */
void orq_release(or_quotas* Q, const ke_pod* pod, int assigned, int del);
#endif
