/*
 * topology.c — which GPU an mTCP core drives, by NUMA node (SURVEY.md §8e:
 * each GPU's batches come from "its own host thread (NUMA-local)").
 *
 * mOS binds every mTCP thread and its memory to the core's node
 * (mtcp_core_affinitize, core/src/cpu.c:56-87, called at core.c:1291 before
 * init_handle at :1313) and DPDK places each port's queues on the port's socket
 * (dpdk_module.c:679, :726-743).  The GPU path does the same: core c drives a
 * GPU attached to c's node -- round robin over that node's GPUs by c's rank
 * among the node's cores -- so the frames it stages cross PCIe from local
 * memory; the staging is allocated by the thread itself after mOS bound it
 * (hipHostMallocNumaUser, mosrx_host_alloc).  Where the topology is not known
 * (no sysfs entry, a GPU without a node) or c's node has no GPU, c drives
 * gpu_base + c % ngpu, the round-3 map.
 *
 * Everything is read from sysfs under a settable root (a fake tree in the CPU
 * tests): /sys/bus/pci/devices/<bdf>/numa_node for a GPU (its PCI address from
 * hipDeviceGetPCIBusId), /sys/devices/system/cpu/cpu<c>/node<n> for a core and
 * /sys/devices/system/node/node<n>/cpulist for the cores of a node.
 */
#define _GNU_SOURCE
#include <ctype.h>
#include <dirent.h>
#include <errno.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>

#include "../../include/mosrx_io_module.h"

static char g_root[512] = "";
static pthread_mutex_t g_topo_lock = PTHREAD_MUTEX_INITIALIZER;

int mosrx_topology_set_root(const char *root)
{
	if (root && strlen(root) >= sizeof(g_root) - 1)
		return -ENAMETOOLONG;
	pthread_mutex_lock(&g_topo_lock);
	snprintf(g_root, sizeof(g_root), "%s", root && strcmp(root, "/") ? root : "");
	pthread_mutex_unlock(&g_topo_lock);
	return 0;
}

static int read_int(const char *path, int *v)
{
	FILE *f = fopen(path, "r");
	int ok;
	if (!f)
		return -1;
	ok = fscanf(f, "%d", v) == 1;
	fclose(f);
	return ok ? 0 : -1;
}

int mosrx_pci_numa_node(const char *bdf)
{
	char path[1024], low[64];
	int v, i;
	if (!bdf || strlen(bdf) >= sizeof(low))
		return -1;
	for (i = 0; bdf[i]; i++)
		low[i] = (char)tolower((unsigned char)bdf[i]);
	low[i] = 0;
	snprintf(path, sizeof(path), "%s/sys/bus/pci/devices/%s/numa_node", g_root, low);
	return read_int(path, &v) ? -1 : v;
}

/* The node of core `cpu`: the cpu<c>/node<n> entry sysfs keeps for it. */
int mosrx_cpu_numa_node(int cpu)
{
	char path[1024];
	DIR *d;
	struct dirent *e;
	int node = -1;
	if (cpu < 0)
		return -1;
	snprintf(path, sizeof(path), "%s/sys/devices/system/cpu/cpu%d", g_root, cpu);
	if (!(d = opendir(path)))
		return -1;
	while ((e = readdir(d)))
		if (!strncmp(e->d_name, "node", 4) && isdigit((unsigned char)e->d_name[4])) {
			node = atoi(e->d_name + 4);
			break;
		}
	closedir(d);
	return node;
}

/* c's position among the cores of `node` (its cpulist, "0-7,16-23" form), -1 if absent. */
static int cpu_rank_in_node(int cpu, int node)
{
	char path[1024], buf[4096], *p;
	FILE *f;
	int rank = 0;
	snprintf(path, sizeof(path), "%s/sys/devices/system/node/node%d/cpulist", g_root, node);
	if (!(f = fopen(path, "r")))
		return -1;
	if (!fgets(buf, sizeof(buf), f)) {
		fclose(f);
		return -1;
	}
	fclose(f);
	for (p = buf; *p && *p != '\n';) {
		char *end;
		long lo = strtol(p, &end, 10), hi;
		if (end == p)
			break;
		hi = lo;
		p = end;
		if (*p == '-') {
			hi = strtol(p + 1, &end, 10);
			p = end;
		}
		if (cpu >= lo && cpu <= hi)
			return rank + (int)(cpu - lo);
		rank += (int)(hi - lo + 1);
		if (*p == ',')
			p++;
	}
	return -1;
}

/* The policy, given the nodes of the candidate GPUs (index 0..ngpu-1): one on
 * c's node, round robin by c's rank among that node's cores; -1 when the
 * topology does not say (the caller then takes c % ngpu). */
int mosrx_numa_pick(int cpu, const int *gpu_node, int ngpu)
{
	int node, rank, i, k, cnt = 0;
	if (cpu < 0 || !gpu_node || ngpu <= 0)
		return -1;
	for (i = 0; i < ngpu; i++)
		if (gpu_node[i] < 0)
			return -1;
	pthread_mutex_lock(&g_topo_lock);
	node = mosrx_cpu_numa_node(cpu);
	rank = node >= 0 ? cpu_rank_in_node(cpu, node) : -1;
	pthread_mutex_unlock(&g_topo_lock);
	if (node < 0 || rank < 0)
		return -1;
	for (i = 0; i < ngpu; i++)
		cnt += gpu_node[i] == node;
	if (!cnt)
		return -1;
	for (i = 0, k = rank % cnt; i < ngpu; i++)
		if (gpu_node[i] == node && k-- == 0)
			return i;
	return -1;
}

int mosrx_gpu_numa_node(int device)
{
	char bdf[64];
	if (hipDeviceGetPCIBusId(bdf, sizeof(bdf), device) != hipSuccess)
		return -1;
	return mosrx_pci_numa_node(bdf);
}
