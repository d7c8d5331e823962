#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
static void hsc(double a, double *so, double *co) {
    const double INV = 6.36619772367581382433e-01;      /* 2/pi */
    const double P1 = 1.5707963267948966192e+00;
    const double P2 = 6.123233995736766036e-17;
    const double P3 = -1.4973849048591698e-33;
    const double n = rint(a * INV);
    const double r1 = fma(-n, P1, a);          /* exact for |n| <= 8 */
    const double w = n * P2;
    const double r = r1 - w;
    const double y = ((r1 - r) - w) - n * P3;  /* tail of r */
    const double z = r * r, v = z * r;
    const double S1=-1.66666666666666324348e-01,S2=8.33333333332248946124e-03,S3=-1.98412698298579493134e-04,
      S4=2.75573137070700676789e-06,S5=-2.50507602534068634195e-08,S6=1.58969099521155010221e-10;
    const double C1=4.16666666666666019037e-02,C2=-1.38888888888741095749e-03,C3=2.48015872894767294178e-05,
      C4=-2.75573143513906633035e-07,C5=2.08757232129817482790e-09,C6=-1.13596475577881948265e-11;
    const double ps = fma(z, fma(z, fma(z, fma(z, S6, S5), S4), S3), S2);
    const double s = r - (fma(z, fma(-v, ps, 0.5 * y), -y) - v * S1);
    const double pc = z * fma(z, fma(z, fma(z, fma(z, fma(z, C6, C5), C4), C3), C2), C1);
    const double hz = 0.5 * z, wc = 1.0 - hz;
    const double c = wc + (((1.0 - wc) - hz) + fma(z, pc, -r * y));
    const int q = ((int)n) & 3;
    double sv = (q & 1) ? c : s, cv = (q & 1) ? s : c;
    if (q == 1 || q == 2) cv = -cv;  /* cos: q=1 -> -sin, q=2 -> -cos */
    if (q == 2 || q == 3) sv = -sv;  /* sin: q=2 -> -sin, q=3 -> -cos */
    *so = sv; *co = cv;
}
static double ulps(double x, double ref) {
    long double e = fabsl((long double)x - (long double)ref);
    double u = nextafter(fabs(ref), INFINITY) - fabs(ref);
    return (double)(e / u);
}
int main() {
    double ms = 0, mc = 0, xs = 0, xc = 0; long cnt = 0, neq = 0;
    srand48(1);
    for (long i = 0; i < 20000000; ++i) {
        double deg = (drand48() * 2 - 1) * 720.0;
        if (i < 2000) deg = (double)(i - 1000) * 0.5;     /* exact multiples of quadrants */
        double a = deg / 180.0 * 3.141592653589793115997963468544185161590576171875;
        double s, c; hsc(a, &s, &c);
        long double rs = sinl((long double)a), rc = cosl((long double)a);
        double es = fabs((double)((s - rs) / (nextafter(fabs((double)rs), INFINITY) - fabs((double)rs))));
        double ec = fabs((double)((c - rc) / (nextafter(fabs((double)rc), INFINITY) - fabs((double)rc))));
        if (es > ms) { ms = es; xs = a; }
        if (ec > mc) { mc = ec; xc = a; }
        if (s != sin(a) || c != cos(a)) neq++;
        cnt++;
    }
    printf("max ulp sin %.3f at %.17g, cos %.3f at %.17g; differs from glibc in %ld of %ld\n", ms, xs, mc, xc, neq, cnt);
    /* glibc's own error vs long double for reference */
    double gs=0,gc=0; srand48(1);
    for (long i = 0; i < 2000000; ++i) { double a=((drand48()*2-1)*720.0)/180.0*3.141592653589793115997963468544185161590576171875;
      long double rs=sinl(a), rc=cosl(a);
      double es=fabs((double)((sin(a)-rs)/(nextafter(fabs((double)rs),INFINITY)-fabs((double)rs))));
      double ec=fabs((double)((cos(a)-rc)/(nextafter(fabs((double)rc),INFINITY)-fabs((double)rc))));
      if(es>gs)gs=es; if(ec>gc)gc=ec; }
    printf("glibc max ulp sin %.3f cos %.3f\n", gs, gc);
}
