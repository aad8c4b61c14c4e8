#include <thread>
#include <vector>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <cstdint>
#include <cstdlib>
int main(){
  const size_t m=720600;
  std::vector<uint32_t> a(m),b(m); std::vector<uint64_t> l(m); std::vector<float> f(m);
  for(size_t i=0;i<m;i++){a[i]=rand()%1200;b[i]=rand()%1200;l[i]=1+rand();f[i]=0.01f;}
  std::vector<char> st(m*20);
  for(int T: {1,2,4,8}){
    double best=1e9;
    for(int rep=0;rep<20;rep++){
      auto t0=std::chrono::steady_clock::now();
      std::vector<std::thread> th; std::vector<uint32_t> bad(T), ns(T);
      auto work=[&](int t){ size_t e0=m*t/T,e1=m*(t+1)/T; uint32_t bd=0,s=0;
        for(size_t e=e0;e<e1;e++){bd|=(a[e]>=1200)|(b[e]>=1200); s+=a[e]==b[e];}
        bad[t]=bd; ns[t]=s;
        memcpy(st.data()+e0*4,a.data()+e0,(e1-e0)*4); memcpy(st.data()+m*4+e0*4,b.data()+e0,(e1-e0)*4);
        memcpy(st.data()+m*8+e0*8,l.data()+e0,(e1-e0)*8); memcpy(st.data()+m*16+e0*4,f.data()+e0,(e1-e0)*4);};
      for(int t=1;t<T;t++) th.emplace_back(work,t);
      work(0);
      for(auto&x:th) x.join();
      double us=std::chrono::duration<double,std::micro>(std::chrono::steady_clock::now()-t0).count();
      if(us<best)best=us;
    }
    printf("T=%d best %.1f us\n",T,best);
  }
}
