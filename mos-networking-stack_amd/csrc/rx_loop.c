/*
 * rx_loop.c — the receive half of RunMainLoop (core.c:897-909) over any
 * io_module_func, consuming the GPU verdicts instead of re-running the checks.
 *
 *   for rx_inf in netdevs:                        core.c:897
 *     recv_cnt = iom->recv_pkts(ctx, rx_inf)      core.c:899
 *     for i < recv_cnt:                           core.c:902
 *       pkt = iom->get_rptr(ctx, rx_inf, i, &len) core.c:905
 *       ProcessPacket(...)                        core.c:906 -> here: NETSTAT + fn()
 *
 * NETSTAT follows eth_in.c:42-45 and :80-84: rx_packets++, rx_bytes += len +
 * ETHER_OVR (24, mtcp.h:58), rx_errors++ when the verdict is negative.
 */
#include <errno.h>
#include <string.h>

#include "../../include/mosrx_io_module.h"

#define ETHER_OVR 24

int mosrx_rx_loop(const io_module_func *iom, struct mtcp_thread_context *ctx, int nif,
                  uint64_t max_pkts, mosrx_pkt_fn fn, void *arg, mosrx_rx_stats *st)
{
	int rx_inf;
	if (!iom || !iom->recv_pkts || !iom->get_rptr || !st || nif <= 0)
		return -EINVAL;
	memset(st, 0, sizeof(*st));
	for (;;) {
		int any = 0;
		st->rounds++;
		for (rx_inf = 0; rx_inf < nif; rx_inf++) {
			const mosrx_result *res = NULL;
			int32_t recv_cnt = iom->recv_pkts(ctx, rx_inf);
			int32_t i;
			if (recv_cnt < 0)
				return -EIO;
			if (recv_cnt == 0)
				continue;
			any = 1;
			st->batches++;
			if (!iom->dev_ioctl || iom->dev_ioctl(ctx, rx_inf, MOSRX_PKT_RX_RESULTS, &res) || !res)
				return -ENOTSUP;   /* the backend must be a classifying one */
			for (i = 0; i < recv_cnt; i++) {
				uint16_t len = 0;
				const uint8_t *pkt = iom->get_rptr(ctx, rx_inf, i, &len);
				const mosrx_result *r = &res[i];
				if (!pkt)
					return -EIO;
				st->rx_packets++;
				st->rx_bytes += (uint64_t)len + ETHER_OVR;
				if (r->verdict < 0)
					st->rx_errors++;
				if (r->reason < MOSRX_R_COUNT)
					st->by_reason[r->reason]++;
				if (fn)
					fn(arg, rx_inf, i, pkt, len, r);
			}
			if (max_pkts && st->rx_packets >= max_pkts)
				return 0;
		}
		if (!any)
			return 0;
	}
}
