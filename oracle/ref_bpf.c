/*
 * ref_bpf.c — TEST INFRASTRUCTURE ONLY.  Driver around mOS's own BPF objects
 * (the core/src/bpf sources, compiled where they lie by `make -C oracle ref`) that
 * produces the golden vectors for the batched BPF row.
 *
 *   mosbpf <exprs.txt> <trace.in> <out.bin>
 *
 * exprs.txt: one filter expression per line, compiled exactly as mOS's
 *   SET_BPFFILTER does: sfbpf_compile(ETH_FRAME_LEN, DLT_EN10MB, &fc, expr, 1, 0)
 *   (include/bpf/sfbpf.h:83, called from mos_api.c:127-155).  A line
 *   "raw:<hex>" is a hand-assembled program instead (8 bytes per insn, the
 *   in-memory struct sfbpf_insn), for interpreter paths no expression emits.
 * trace.in:  u32 n, u32 frames_bytes, n x u32 off, n x u16 len, frames bytes.
 * out.bin, per expression:
 *   i32 compile_rc, i32 validate, u32 ninsn, ninsn x {u16 code, u8 jt, u8 jf, u32 k},
 *   (the two result arrays are 0 when compile_rc < 0 or validate == 0)
 *   n x u32 ret_frame  = sfbpf_filter(insns, frame, caplen, caplen)
 *                        (EVAL_BPFFILTER on ethh/eth_len, ip_in.c:56-63)
 *   n x u32 ret_ip     = sfbpf_filter(insns, frame, 14 + ip_len, 14 + ip_len)
 *                        (EVAL_BPFFILTER on iph - 14 / ip_len + 14, tcp.c:49-52, 486-496)
 *                        for IPv4 frames whose datagram lies inside caplen, else 0.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sfbpf.h"
#include "sfbpf_dlt.h"

#ifndef ETH_FRAME_LEN
#define ETH_FRAME_LEN 1514
#endif

static void *slurp(const char *path, size_t *sz)
{
	FILE *f = fopen(path, "rb");
	void *b;
	if (!f)
		return NULL;
	fseek(f, 0, SEEK_END);
	*sz = (size_t)ftell(f);
	fseek(f, 0, SEEK_SET);
	b = malloc(*sz + 1);
	if (b && fread(b, 1, *sz, f) != *sz) {
		free(b);
		b = NULL;
	}
	fclose(f);
	return b;
}

int main(int argc, char **argv)
{
	size_t esz, tsz;
	char *exprs, *line, *save = NULL;
	uint8_t *tr, *frames;
	uint32_t n, fb, i;
	uint32_t *off;
	uint16_t *len;
	FILE *out;

	if (argc != 4)
		return 2;
	exprs = slurp(argv[1], &esz);
	tr = slurp(argv[2], &tsz);
	if (!exprs || !tr)
		return 1;
	exprs[esz] = 0;
	memcpy(&n, tr, 4);
	memcpy(&fb, tr + 4, 4);
	off = (uint32_t *)(tr + 8);
	len = (uint16_t *)(tr + 8 + 4 * (size_t)n);
	frames = tr + 8 + 6 * (size_t)n;
	out = fopen(argv[3], "wb");
	if (!out)
		return 1;
	for (line = strtok_r(exprs, "\n", &save); line; line = strtok_r(NULL, "\n", &save)) {
		struct sfbpf_program fc;
		int32_t rc, val = 0;
		uint32_t ninsn = 0;
		memset(&fc, 0, sizeof(fc));
		if (!strncmp(line, "raw:", 4)) {
			size_t nb = strlen(line + 4) / 2, b;
			uint8_t *ins = calloc(nb + 8, 1);
			for (b = 0; b < nb; b++) {
				unsigned v;
				sscanf(line + 4 + 2 * b, "%2x", &v);
				ins[b] = (uint8_t)v;
			}
			fc.bf_len = (unsigned)(nb / 8);
			fc.bf_insns = (struct sfbpf_insn *)ins;
			rc = 0;
		} else {
			rc = sfbpf_compile(ETH_FRAME_LEN, DLT_EN10MB, &fc, line, 1, 0);
		}
		if (rc >= 0) {
			ninsn = fc.bf_len;
			val = sfbpf_validate(fc.bf_insns, (int)fc.bf_len);
		}
		fwrite(&rc, 4, 1, out);
		fwrite(&val, 4, 1, out);
		fwrite(&ninsn, 4, 1, out);
		if (ninsn)
			fwrite(fc.bf_insns, 8, ninsn, out);
		for (i = 0; i < n; i++) {
			uint32_t r = 0;
			if (rc >= 0 && val && off[i] + (uint64_t)len[i] <= fb)
				r = sfbpf_filter(fc.bf_insns, frames + off[i], len[i], len[i]);
			fwrite(&r, 4, 1, out);
		}
		for (i = 0; i < n; i++) {
			uint32_t r = 0;
			const uint8_t *f = frames + off[i];
			if (rc >= 0 && val && off[i] + (uint64_t)len[i] <= fb && len[i] >= 18 && f[12] == 0x08 && f[13] == 0x00) {
				uint32_t l = 14u + ((uint32_t)f[16] << 8 | f[17]);
				if (l <= len[i])
					r = sfbpf_filter(fc.bf_insns, f, l, l);
			}
			fwrite(&r, 4, 1, out);
		}
		if (rc >= 0 && !strncmp(line, "raw:", 4))
			free(fc.bf_insns);
		else if (rc >= 0)
			sfbpf_freecode(&fc);
	}
	fclose(out);
	return 0;
}
