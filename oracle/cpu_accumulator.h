/* Oracle (test infrastructure only): the CPU accumulator restatement, see cpu_accumulator.c. */
#ifndef KE_ORACLE_CPU_ACCUMULATOR_H
#define KE_ORACLE_CPU_ACCUMULATOR_H
#include <stdint.h>

#define ACC_MAX_CPUS 256 /* CPU ids 0..255 */
#define ACC_WORDS (ACC_MAX_CPUS / 64)
#define ACC_EXCL_NONE 0 /* CPUExclusivePolicy */
#define ACC_EXCL_PCPU 1
#define ACC_EXCL_NUMA 2
#define ACC_BIND_NONE 0 /* CPUBindPolicy */
#define ACC_BIND_FULL_PCPUS 1
#define ACC_BIND_SPREAD_BY_PCPUS 2

/* CPUTopology: per CPU id its core / NUMA node / socket ids as the reference holds them */
typedef struct acc_topo {
  uint8_t valid[ACC_MAX_CPUS];
  int core[ACC_MAX_CPUS], node[ACC_MAX_CPUS], socket[ACC_MAX_CPUS];
  int num_cpus, num_cores, num_nodes, num_sockets;
} acc_topo;

/* the allocated CPUs' CPUDetails (RefCount, ExclusivePolicy) */
typedef struct acc_alloc {
  uint8_t present[ACC_MAX_CPUS];
  int ref[ACC_MAX_CPUS];
  int excl[ACC_MAX_CPUS];
} acc_alloc;

void acc_topo_finish(acc_topo* t);
int acc_cpus_per_core(const acc_topo* t);
int acc_cpus_per_socket(const acc_topo* t);
int acc_cpus_per_node(const acc_topo* t);
int acc_take_cpus(const acc_topo* t, int max_ref, const uint64_t* available, const acc_alloc* allocated, int needed,
                  int bind, int excl_policy, int numa_most, uint64_t* result);
int acc_take_preferred_cpus(const acc_topo* t, int max_ref, const uint64_t* available, const uint64_t* preferred,
                            const acc_alloc* allocated, int needed, int bind, int excl_policy, int numa_most,
                            uint64_t* result);
int acc_spread_order(const acc_topo* t, const uint64_t* available, int numa_most, int* out);
#endif
