/* Ray-mix statistics of C3 (final scene, 1200x800, depth 50) from the C oracle:
 * classes of the traced rays (the device ends a sample at its first C == 0
 * origin). Analysis only.
 *   gcc -O2 -ffp-contract=off -Ioracle -o /tmp/raymix tests/models/raymix.c -lm -lpthread && /tmp/raymix 20000 */
#include "../oracle/rt_oracle.c"
#include <stdio.h>
static double Cof(const rt_sphere* s, const double o[3]) {
  double ax=o[0]-s->cx, ay=o[1]-s->cy, az=o[2]-s->cz;
  return ((ax*ax+ay*ay)+az*az) - s->r*s->r;
}
int main(int argc, char** argv) {
  rt_sphere sph[600]; int n = oracle_scene_random_spheres(1, sph, 600);
  rt_camera cam; double from[3]={13,2,3}, at[3]={0,0,0}, up[3]={0,1,0};
  oracle_camera_look_at(from, at, up, 20.0, 1200.0/800.0, &cam);
  rt_params p; memset(&p,0,sizeof p); p.width=1200; p.height=800; p.spp=100; p.max_depth=50; p.seed=0;
  oracle_bounce tr[64];
  long N = argc>1 ? atol(argv[1]) : 20000;
  uint64_t x = 12345;
  long cls[16]={0}; long traced=0, samples=0, trapped=0;
  long crawl_Cneg=0, crawl_Cpos=0, crawl_Czero=0, crawl_same_o=0, crawl_front=0;
  long after_crawl[8]={0};
  long hist_len[64]={0};
  for (long it=0; it<N; ++it) {
    x = x*6364136223846793005ULL+1442695040888963407ULL;
    int i = (x>>33)%1200, j=(x>>13)%800, s=(x>>50)%100;
    double col[3];
    int len = oracle_trace_sample(sph, n, &cam, &p, i, j, s, col, tr, 64);
    samples++;
    int prev=-1;
    int L = len;
    // emulate trap: at ray k (k>=1) origin on hint sphere prev with C==0 -> stop
    for (int k=0;k<len;k++){
      if (k>=1) {
        int h = tr[k-1].index;
        if (h>=0 && Cof(&sph[h], tr[k].o)==0.0) { trapped++; L=k+1; break; }
      }
    }
    traced += L; hist_len[L<63?L:63]++;
    for (int k=0;k<L;k++){
      int c;
      if (k==0) c=0;
      else {
        int h=tr[k-1].index;
        if (tr[k].index<0) c=1;
        else if (tr[k].index==h && tr[k].t<1e-6) c=2;
        else if (tr[k].index==h) c=3;
        else c=4;
        if (c==2) {
          double C=Cof(&sph[h], tr[k].o);
          if (C<0) crawl_Cneg++; else if (C>0) crawl_Cpos++; else crawl_Czero++;
          if (tr[k-1].front_face) crawl_front++;
          if (k+1<L) { int c2; if (tr[k+1].index<0) c2=1; else if (tr[k+1].index==h && tr[k+1].t<1e-6) c2=2; else if (tr[k+1].index==h) c2=3; else c2=4; after_crawl[c2]++; }
          else after_crawl[0]++;
          double *o1=tr[k].o; 
          if (k+1<len && tr[k+1].o[0]==o1[0]&&tr[k+1].o[1]==o1[1]&&tr[k+1].o[2]==o1[2]) crawl_same_o++;
        }
      }
      cls[c]++;
    }
  }
  printf("samples %ld traced %ld (%.3f/sample) trapped %ld\n", samples, traced, (double)traced/samples, trapped);
  const char* nm[]={"camera","miss","crawl(same,t<1e-6)","same sphere chord","other sphere"};
  for(int c=0;c<5;c++) printf("%-22s %ld %.3f\n", nm[c], cls[c], (double)cls[c]/traced);
  printf("crawl: C<0 %ld C>0 %ld C==0 %ld prevfront %ld nextorigin==o %ld\n", crawl_Cneg, crawl_Cpos, crawl_Czero, crawl_front, crawl_same_o);
  printf("after crawl: end %ld miss %ld crawl %ld chord %ld other %ld\n", after_crawl[0], after_crawl[1], after_crawl[2], after_crawl[3], after_crawl[4]);
  for (int l=0;l<64;l++) if(hist_len[l]) printf("len %d: %ld\n", l, hist_len[l]);
}
