/* mosrx_source.h — internal: the frame-source vtable behind mosrx_source_* */
#ifndef MOSRX_SOURCE_H
#define MOSRX_SOURCE_H

#include <stdint.h>

struct mosrx_source {
	/* write the next frame into dst (at most cap bytes); returns its caplen, 0 when none */
	int  (*next)(struct mosrx_source *s, uint8_t *dst, uint32_t cap);
	void (*close)(struct mosrx_source *s);
};

#endif
