#define CHR_SOURCE_SHA "8fc66f2cbf19b283"
