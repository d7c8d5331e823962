/* Check (CPU) that deg2rad's division-free a / 180 in csrc/hpe_device.hpp returns the
 * correctly rounded quotient bit for bit: 2e9 random doubles of every significand with
 * exponents 2^-10..2^10 (both signs; the angles the FK sees lie within +-540) plus every
 * multiple of 1/1000 and every integer in +-360.  Build: gcc -O2 -ffp-contract=off
 * tools/div180_check.c -lm.  (Markstein's theorem gives it for all finite a without
 * underflow: y = RN(1/180), q0 = RN(a y) faithful, r = a - 180 q0 exact, RN(q0 + r y).) */
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <math.h>
static inline double div180(double a){ const double y=1.0/180.0; double q0=a*y; double r=fma(-q0,180.0,a); double q=fma(r,y,q0); return a==0.0? a : q; }
static uint64_t s=88172645463325252ull; static inline uint64_t xr(){ s^=s<<13; s^=s>>7; s^=s<<17; return s; }
int main(){ uint64_t bad=0, n=0;
 // every double in [2^-10, 1024) sampled by random bit patterns of the significand, both signs
 for (long i=0;i<2000000000L;i++){ uint64_t b=xr(); int e=(int)(b>>52)&0x7ff; e = 1023-10 + (e % 21); // exponents 2^-10..2^10
   uint64_t bits = ((uint64_t)e<<52) | (b & 0xfffffffffffffull) | ((b>>63)<<63); double a; memcpy(&a,&bits,8);
   double r1=a/180.0, r2=div180(a); n++; if (memcmp(&r1,&r2,8)) { if (bad<5) printf("mismatch %.17g: %.17g %.17g\n",a,r1,r2); bad++; } }
 // integers and common decimal angles
 for (long k=-360000;k<=360000;k++){ double a=k/1000.0; double r1=a/180.0, r2=div180(a); n++; if (memcmp(&r1,&r2,8)) bad++; a=(double)k; r1=a/180.0; r2=div180(a); n++; if (memcmp(&r1,&r2,8)) bad++; }
 printf("checked %llu, mismatches %llu\n",(unsigned long long)n,(unsigned long long)bad); return bad!=0; }
