/* host build: nothing from this header is used by mislo_probe.h */
